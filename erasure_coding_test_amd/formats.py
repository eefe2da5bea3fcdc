"""Wire and disk formats either side of the coding path.

The reference's client and datanodes exchange raw ``metadata_t`` structs and
store each shard ("chunk") of a stripe as one file per datanode.  This module
restates those formats so a host program around the GPU coding path reads and
writes exactly the bytes the reference's programs do:

* ``metadata_t`` (``include/ych_ec_test.h:47-61``) -- sent as its raw x86-64
  in-memory image, ``send(fd, metadata, sizeof(metadata_t))``
  (``client_main.cpp:153``, ``:564``, ``:865``), 312 bytes in the reference's
  default build (``ENCODE_ISOMERISM_MODE 1``, ``EC_X 3``);
* chunk file names ``<dst><stripe>_<idx+1>`` (``client_main.cpp:1366``, ``:253``);
* the file-size sidecar: ``"%d"`` in a zeroed 256-byte buffer, written and read
  whole (``client_main.cpp:1886-1890``, ``:2001-2015``);
* the ``'0'`` (0x30) padding of a short read (``client_main.cpp:31-53``);
* the read path's tail arithmetic (``client_main.cpp:2017-2026``, ``:2150-2178``);
* the ECK/ECX block split of a chunk (``client_main.cpp:1450-1451``, ``:1463-1476``)
  and the byte offset each block lands at on disk (``eck_datanode_main.cpp:442-470``,
  ``ecx_datanode_main.cpp:793-822``), and which ECX datanode encodes which block
  (``ecx_datanode_main.cpp:1494-1495``, ``:1114-1117``).

Pure host code: no GPU, no sockets.  ``tests/cluster_replay.py`` drives these
formats over 127.0.7.x sockets to replay client <-> ECK <-> ECX on one host.
"""
from __future__ import annotations

import ctypes
from typing import BinaryIO, Dict, List, Optional, Tuple

# ych_ec_test.h:1-46 (the reference's default build)
EC_K, EC_M, EC_W = 3, 3, 8
CHUNK_SIZE_MB = 1
EC_X, EC_N = 3, 3
TEST_N = 3
MAX_PATH_LEN = 256
EC_ERROR, EC_OK = -1, 0
IP_PREFIX = "192.168.7."
DATANODE_START_IP_ADDR = 102
EC_WRITE_PORT = 8000
EC_READ_PORT = 8001
EC_WRITE_NEW_PORT = 8002
EC_WRITE_ECK_BASE_PORT = 8010
EC_WRITE_ECX_BASE_PORT = 8050
EC_WRITE_REQUEST_BASE_PORT = 8090
WRITE_PATH = "test_file/write/"
READ_PATH = "test_file/read/"
FILE_SIZE_PATH = "test_file/file_size/file_size_"
PAD_BYTE = b"0"  # client_main.cpp:49 pads with the character '0', not NUL


def metadata_struct(ec_x: int = EC_X, net_block_size: bool = True) -> type:
    """ctypes image of ``metadata_t`` (ych_ec_test.h:47-61).

    ``net_block_size[EC_X]`` exists only when NET_BANDWIDTH_MODE or
    ENCODE_ISOMERISM_MODE is set (ych_ec_test.h:57-59); the reference's default
    build has it with EC_X = 3, giving 312 bytes.  Natural x86-64 alignment, as
    gcc lays the struct out."""
    fields = [
        ("sockfd", ctypes.c_int),
        ("chunk_size", ctypes.c_long),          # chunk size, or the block's file offset
        ("block_size", ctypes.c_int),           # -1 marks a whole chunk (client_main.cpp:625)
        ("remain_block_size", ctypes.c_int),
        ("cur_block", ctypes.c_int),
        ("cur_eck", ctypes.c_int),
        ("data", ctypes.c_void_p),              # sender's pointer, meaningless to the receiver
        ("dst_filename_datanode", ctypes.c_char * MAX_PATH_LEN),
        ("error_flag", ctypes.c_int),
    ]
    if net_block_size:
        fields.append(("net_block_size", ctypes.c_int * ec_x))

    class metadata_t(ctypes.Structure):
        _fields_ = fields

    return metadata_t


MetadataT = metadata_struct()
METADATA_SIZE = ctypes.sizeof(MetadataT)


def pack_metadata(*, sockfd: int = 0, chunk_size: int = 0, block_size: int = 0, remain_block_size: int = 0,
                  cur_block: int = 0, cur_eck: int = 0, data: int = 0, dst_filename_datanode: str = "",
                  error_flag: int = EC_OK, net_block_size: Optional[List[int]] = None,
                  struct: type = MetadataT) -> bytes:
    """Raw bytes of one ``metadata_t``.  Fields the reference leaves
    uninitialised on the stack (e.g. ``remain_block_size`` in
    ``send_chunks_datanodes``) are zero here; receivers never read them."""
    name = dst_filename_datanode.encode()
    if len(name) >= MAX_PATH_LEN:
        raise ValueError(f"dst_filename_datanode longer than {MAX_PATH_LEN - 1} bytes (sprintf would overflow)")
    md = struct()
    md.sockfd, md.chunk_size, md.block_size = sockfd, chunk_size, block_size
    md.remain_block_size, md.cur_block, md.cur_eck = remain_block_size, cur_block, cur_eck
    md.data, md.dst_filename_datanode, md.error_flag = data or None, name, error_flag
    if net_block_size is not None:
        if not hasattr(md, "net_block_size") or len(net_block_size) != len(md.net_block_size):
            raise ValueError("net_block_size does not match the struct's EC_X")
        for i, v in enumerate(net_block_size):
            md.net_block_size[i] = v
    return bytes(md)


def unpack_metadata(raw: bytes, struct: type = MetadataT) -> Dict[str, object]:
    if len(raw) != ctypes.sizeof(struct):
        raise ValueError(f"metadata_t is {ctypes.sizeof(struct)} bytes, got {len(raw)}")
    md = struct.from_buffer_copy(raw)
    out = {name: getattr(md, name) for name, _ in struct._fields_}
    out["data"] = md.data or 0
    out["dst_filename_datanode"] = md.dst_filename_datanode.decode(errors="surrogateescape")
    if "net_block_size" in out:
        out["net_block_size"] = list(md.net_block_size)
    return out


# ---- names ----------------------------------------------------------------

def stripe_filename(dst_filename: str, stripe: int) -> str:
    """``dst_filename_stripe``: ``sprintf("%s%d", dst_filename, current_reading)``
    with the 1-based stripe number (client_main.cpp:1366, :2060)."""
    return f"{dst_filename}{stripe}"


def chunk_filename(dst_filename_stripe: str, idx: int) -> str:
    """Chunk ``idx`` (0-based: data 0..k-1, coding k..k+m-1) of a stripe on its
    datanode: ``sprintf("%s_%d", dst_filename_stripe, i + 1)`` (client_main.cpp:253)."""
    name = f"{dst_filename_stripe}_{idx + 1}"
    if len(name.encode()) >= MAX_PATH_LEN:
        raise ValueError(f"chunk file name longer than {MAX_PATH_LEN - 1} bytes")
    return name


def datanode_ip(idx: int, prefix: str = IP_PREFIX, start: int = DATANODE_START_IP_ADDR) -> str:
    """Address of datanode ``idx`` (client_main.cpp:72); idx -1 is the client (ECK/ECX
    ``initialize_network(..., -1)`` reaches it for chunk_ok, eck_datanode_main.cpp:252)."""
    return f"{prefix}{start + idx}"


# ---- file size sidecar ----------------------------------------------------

def file_size_sidecar(file_size: int) -> bytes:
    """The bytes written to ``FILE_SIZE_PATH<dst>``: ``sprintf(buf, "%d", file_size)``
    into a zeroed ``char[MAX_PATH_LEN]`` and ``fwrite`` of the whole buffer
    (client_main.cpp:1888-1889).  ``int`` in the reference: sizes >= 2 GiB wrap."""
    if not -2 ** 31 <= file_size < 2 ** 31:
        raise ValueError("file_size does not fit the reference's int")
    text = b"%d" % file_size
    return text + bytes(MAX_PATH_LEN - len(text))


def parse_file_size_sidecar(raw: bytes) -> int:
    """``fread`` of exactly MAX_PATH_LEN bytes then ``atoi`` (client_main.cpp:2008-2015):
    a short sidecar is an error; atoi stops at the first non-digit."""
    if len(raw) != MAX_PATH_LEN:
        raise ValueError(f"file size sidecar must be {MAX_PATH_LEN} bytes, got {len(raw)}")
    s = raw.split(b"\0", 1)[0].lstrip(b" \t\n\r\f\v")
    sign, i = 1, 0
    if s[:1] in (b"+", b"-"):
        sign, i = (-1 if s[:1] == b"-" else 1), 1
    j = i
    while j < len(s) and 0x30 <= s[j] <= 0x39:
        j += 1
    return sign * int(s[i:j]) if j > i else 0


# ---- stripes over a file --------------------------------------------------

def read_file_to_buffer(f: BinaryIO, buffer: bytearray) -> int:
    """client_main.cpp:31-53: fill ``buffer`` from ``f``; a short read pads the rest
    with '0' (0x30) and returns 0 ("padding read"), a full read returns 1."""
    n = len(buffer)
    got = f.readinto(memoryview(buffer)) or 0
    if got < n:
        buffer[got:] = PAD_BYTE * (n - got)
        return 0
    return 1


def stripe_count(file_size: int, k: int, chunk_size: int) -> int:
    """``reading``: stripes needed for the file (client_main.cpp:1681-1688, :2034-2041)."""
    buffer_size = k * chunk_size
    return file_size // buffer_size + (1 if file_size % buffer_size else 0)


def read_tail(file_size: int, k: int, chunk_size: int) -> Tuple[int, int]:
    """(remain_chunks, remain_size) of the last stripe on the read path
    (client_main.cpp:2017-2026): whole data chunks, then a partial one.  A file
    that fills its last stripe exactly gives (k, 0)."""
    buffer_size = k * chunk_size
    if file_size % buffer_size == 0:
        return k, 0
    r = file_size % buffer_size
    return r // chunk_size, r % chunk_size


def last_stripe_bytes(data_chunks: List[bytes], remain_chunks: int, remain_size: int) -> bytes:
    """What the read path appends for the last stripe (client_main.cpp:2161-2178):
    ``remain_chunks`` whole chunks, then ``remain_size`` bytes of the next."""
    out = b"".join(bytes(c) for c in data_chunks[:remain_chunks])
    if remain_size:
        out += bytes(data_chunks[remain_chunks][:remain_size])
    return out


# ---- ECK / ECX block pipeline --------------------------------------------

def eck_block_sizes(chunk_size: int, w: int = EC_W, n: int = EC_N) -> Tuple[int, int]:
    """(block_size, remain_block_size) for the ``-kw`` write (client_main.cpp:1450-1451):
    whole w-bit words split over ``n`` blocks, the remainder words going to block 0.
    A chunk that is not whole words loses its trailing bytes (never sent)."""
    wb = w // 8
    return ((chunk_size // wb) // n) * wb, ((chunk_size // wb) % n) * wb


def eck_blocks(chunk_size: int, w: int = EC_W, n: int = EC_N) -> List[Tuple[int, int]]:
    """(offset, size) of each of the ``n`` blocks of a chunk: block 0 starts at 0 and
    carries the remainder, block j > 0 starts at remain + j*block_size
    (client_main.cpp:1463-1476, :426-433); the same offsets are where the blocks land
    in the chunk files (``save_offset``, eck_datanode_main.cpp:442-449)."""
    bs, rem = eck_block_sizes(chunk_size, w, n)
    return [(0, bs + rem)] + [(rem + j * bs, bs) for j in range(1, n)]


def ecx_node_for_block(cur_block: int, k: int = EC_K, ec_x: int = EC_X) -> int:
    """Datanode index (k..k+EC_X-1) of the ECX node that encodes block ``cur_block``:
    ECK forwards on ``sockfd_array[cur_block % EC_X]`` (eck_datanode_main.cpp:328),
    connected to datanode EC_K + i (:401)."""
    return k + cur_block % ec_x


def ecx_blocks(ecm: int, k: int = EC_K, n: int = EC_N, ec_x: int = EC_X) -> List[int]:
    """Blocks ECX datanode ``ecm`` encodes, in order: from ``ecm - EC_K`` in steps of
    EC_X (ecx_datanode_main.cpp:1494-1495, :1114-1117); within a block, the k ECK
    sources arrive in order 0..k-1 (the ``cur_eck_net`` gate, :1083-1086)."""
    return list(range(ecm - k, n, ec_x))


def block_offset(cur_block: int, block_size: int, remain_block_size: int,
                 net_block_size: Optional[List[int]] = None) -> int:
    """``save_offset`` of a received block in its chunk file.  Plain build:
    ``remain + cur_block * block_size`` (eck_datanode_main.cpp:442-450).  With
    NET_BANDWIDTH_MODE / ENCODE_ISOMERISM_MODE (the reference's default build) the
    offset is summed from ``net_block_size[]`` instead (:451-471): full rounds of
    EC_X blocks, then the first ``cur_block % EC_X`` entries.  Senders that fill
    ``net_block_size`` with ``block_size`` everywhere get the same offset either way."""
    if cur_block == 0:
        return 0
    if net_block_size is None:
        return remain_block_size + cur_block * block_size
    x = len(net_block_size)
    rounds, rest = divmod(cur_block, x)
    return remain_block_size + sum(net_block_size) * rounds + sum(net_block_size[:rest])


def replace_filename_suffix(filename: str, suffix: int) -> str:
    """ecx_datanode_main.cpp:52-71: replace what follows the last '_' with ``suffix``
    -- how an ECX node turns an ECK chunk name ``<stripe>_<eck+1>`` into its own coding
    chunk name ``<stripe>_<ecm+1>`` (:152).  No '_' is an error (EC_ERROR there)."""
    pos = filename.rfind("_")
    if pos < 0:
        raise ValueError(f"replace_filename_suffix: no '_' in {filename!r}")
    return f"{filename[:pos + 1]}{suffix}"
