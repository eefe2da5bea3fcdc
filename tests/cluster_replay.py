"""Localhost replay of the reference's client <-> ECK <-> ECX programs (TEST INFRASTRUCTURE).

SURVEY.md §8f row 4: the reference's datanodes bind fixed 192.168.7.102+
addresses (ych_ec_test.h:35-36), so its programs cannot run on one host.  This
harness replays their wire protocol and disk layout over 127.0.7.x loopback
addresses (datanode i on 127.0.7.(102+i), the client on 127.0.7.101, the
reference's ports plus an offset) with a pluggable coder, so a test can push
a file through the coding path exactly as the reference's cluster would and
compare every chunk file and the read-back file byte for byte:

* ``-w``  ``Client.write``      -> k data + m coding chunks, one ``metadata_t``
  (block_size = -1) + chunk per datanode (client_main.cpp:607-678, 1590-1918;
  datanode side eck_datanode_main.cpp:545-614, 286-314);
* ``-r``  ``Client.read``       -> data chunks from the k data nodes, a dead node
  becomes an erasure, coding chunks fetched as the reference does, decode,
  tail trimmed by the file-size sidecar (client_main.cpp:860-1046, 1920-2195;
  eck_datanode_main.cpp:694-744);
* ``-kw`` ``Client.write_eck``  -> every data chunk split into EC_N blocks sent
  to the k ECK nodes, which store them at their offsets and forward block j to
  ECX node k + j % EC_X; that node accumulates the m coding blocks of block j
  source by source (ECX incremental encode, ecx_datanode_main.cpp:667-735),
  keeps its own row and ships the others to their coding nodes; every node sends
  chunk_ok to the client after its EC_N blocks (client_main.cpp:381-557,
  eck_datanode_main.cpp:180-285, 315-543, ecx_datanode_main.cpp:1056-1146).
  The reference ships the other coding rows along an ECX->ECX request ring
  (:838-1054); the replay sends them straight to their owners -- same bytes on
  disk, same chunk_ok count.

The metadata on the wire is the reference's raw struct
(``erasure_coding_test_amd.formats``); ints answer as 4-byte native ints with
the reference's polarity (metadata ack 1 = ok, data ack 0 = ok).  Chunk names
are sent relative (``test_file/write/<dst><stripe>_<i>``) and stored under each
node's own directory (the reference's nodes are separate machines sharing one
path layout).  A node acks a chunk after writing it (the reference acks first and
writes from an IO thread), so a finished client call means files on disk.
ENCODE_ISOMERISM's unequal block sizes (``-enckw``) and its
sleep-based delay emulation are not replayed; ``-kw`` fills ``net_block_size``
with the uniform block size, which makes both of the reference's offset
formulas agree (``formats.block_offset``).
"""
from __future__ import annotations

import os
import socket
import struct
import threading
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from erasure_coding_test_amd import formats as F

INT = struct.Struct("=i")
TIMEOUT_S = 30.0


# ---- sockets ---------------------------------------------------------------

def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    view, got = memoryview(buf), 0
    while got < n:
        r = s.recv_into(view[got:], n - got)
        if r == 0:
            raise ConnectionError(f"peer closed after {got} of {n} bytes")
        got += r
    return bytes(buf)


def _send_int(s, v):
    s.sendall(INT.pack(v))


def _recv_int(s) -> int:
    return INT.unpack(_recv_exact(s, INT.size))[0]


def _listen(addr: str, port: int) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind((addr, port))
    s.listen(64)
    s.settimeout(0.2)
    return s


def _connect(addr: str, port: int, src: Optional[str] = None) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.settimeout(TIMEOUT_S)
    if src:
        s.bind((src, 0))
    s.connect((addr, port))
    return s


def _send_metadata_and(s, md: bytes, payload: bytes) -> None:
    """Client/ECK sender side (client_main.cpp:148-195, :559-605)."""
    s.sendall(md)
    if _recv_int(s) == 0:
        raise RuntimeError("metadata rejected (reference: error_response == 0)")
    s.sendall(payload)
    if _recv_int(s) == 1:
        raise RuntimeError("data rejected (reference: error_response == 1)")


# ---- coders ----------------------------------------------------------------

class Coder:
    """What the replay needs from an erasure-coding library."""

    def coding_matrix(self, k: int, m: int, w: int) -> List[int]: ...
    def encode(self, k, m, w, matrix, data, coding, size) -> None: ...
    def decode(self, k, m, w, matrix, erasures, data, coding, size) -> int: ...
    def accumulator(self, m: int, size: int): ...


class ProductCoder(Coder):
    """The product: the GPU path through the package's reference-shaped API."""

    def __init__(self):
        import erasure_coding_test_amd as ec
        self.ec = ec

    def coding_matrix(self, k, m, w):
        return self.ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)

    def encode(self, k, m, w, matrix, data, coding, size):
        self.ec.jerasure.jerasure_matrix_encode(k, m, w, matrix, data, coding, size)

    def decode(self, k, m, w, matrix, erasures, data, coding, size):
        return self.ec.jerasure.jerasure_matrix_decode(k, m, w, matrix, 0, erasures, data, coding, size)

    def accumulator(self, m, size):
        return self.ec.ParityAccumulator(m, size)


class _HostAccumulator:
    """The reference's ECX loop (ecx_datanode_main.cpp:687-735) on the checker."""

    def __init__(self, oracle, m, size):
        self.o, self.m, self.size = oracle, m, size
        self.acc = [np.zeros(size + 8, np.uint8) for _ in range(m)]  # +8: the reference's padding (:684)
        self.init = [0] * m

    def add(self, block, coefs):
        for i, c in enumerate(coefs):
            if c == 1:
                if not self.init[i]:
                    self.acc[i][:self.size] = block[:self.size]
                    self.init[i] = 1
                else:
                    self.o.region_xor(block, self.acc[i], self.acc[i], self.size)
            elif c != 0:
                self.o.region_multiply(block, c, self.size, self.acc[i], self.init[i])
                self.init[i] = 1

    def read(self, i, out, nbytes=-1):
        n = self.size if nbytes < 0 else nbytes
        out[:n] = self.acc[i][:n]
        return bool(self.init[i])

    def reset(self):
        self.init = [0] * self.m


class OracleCoder(Coder):
    """The checker (oracle/): CPU restatement of the reference's w=8 path."""

    def __init__(self, oracle=None):
        if oracle is None:
            from oracle.oracle import Restatement
            oracle = Restatement()
        self.o = oracle

    def coding_matrix(self, k, m, w):
        assert w == 8
        return [int(v) for v in np.asarray(self.o.vandermonde_coding_matrix(k, m)).ravel()]

    def encode(self, k, m, w, matrix, data, coding, size):
        self.o.matrix_encode(k, m, np.asarray(matrix, np.int32), data, coding, size)

    def decode(self, k, m, w, matrix, erasures, data, coding, size):
        return self.o.matrix_decode(k, m, np.asarray(matrix, np.int32), 0, list(erasures), data, coding, size)

    def accumulator(self, m, size):
        return _HostAccumulator(self.o, m, size)


# ---- cluster -----------------------------------------------------------------

class Layout:
    def __init__(self, k=F.EC_K, m=F.EC_M, w=F.EC_W, chunk_size=F.CHUNK_SIZE_MB << 20, ec_x=F.EC_X,
                 ec_n=F.EC_N, port_offset=0, prefix="127.0.7.", start=F.DATANODE_START_IP_ADDR):
        if not 1 <= ec_x <= m or ec_n < ec_x:
            raise ValueError("the reference needs 1 <= EC_X <= EC_M and EC_N >= EC_X (ych_ec_test.h:9-10)")
        self.k, self.m, self.w, self.chunk_size, self.ec_x, self.ec_n = k, m, w, chunk_size, ec_x, ec_n
        self.off, self.prefix, self.start = port_offset, prefix, start
        self.struct = F.metadata_struct(ec_x)
        self.md_size = F.ctypes.sizeof(self.struct)

    def ip(self, idx: int) -> str:
        return F.datanode_ip(idx, self.prefix, self.start)

    def port(self, base: int) -> int:
        return base + self.off

    def pack(self, **kw) -> bytes:
        return F.pack_metadata(struct=self.struct, **kw)

    def unpack(self, raw: bytes) -> dict:
        return F.unpack_metadata(raw, self.struct)


class Datanode:
    """One datanode: ECK behaviour for idx < k, ECX/coding behaviour for idx >= k
    (a coding node also answers plain -w / -r traffic, as both reference programs do)."""

    def __init__(self, L: Layout, idx: int, root: str, coder: Coder, matrix: List[int]):
        self.L, self.idx, self.root, self.coder, self.matrix = L, idx, root, coder, matrix
        self.addr = L.ip(idx)
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._socks: List[socket.socket] = []
        self._io = threading.Lock()
        self._count: Dict[str, int] = {}
        self.errors: List[BaseException] = []
        if idx >= L.k and idx - L.k < L.ec_x:  # an ECX node: the block pipeline state
            self.ecm = idx
            self._gate = threading.Condition()
            self._next = (0, idx - L.k)  # (cur_eck_net, cur_block_net), ecx_datanode_main.cpp:1495
            self._acc = None

    # -- plumbing
    def path(self, name: str) -> str:
        p = os.path.join(self.root, f"node{self.idx}", name.lstrip("/"))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        return p

    def _serve(self, port: int, handler: Callable[[socket.socket], None]) -> None:
        ls = _listen(self.addr, port)
        self._socks.append(ls)

        def loop():
            while not self._stop.is_set():
                try:
                    c, _ = ls.accept()
                except socket.timeout:
                    continue
                except OSError:
                    return
                c.settimeout(TIMEOUT_S)
                t = threading.Thread(target=self._guard, args=(handler, c), daemon=True)
                t.start()

        t = threading.Thread(target=loop, daemon=True)
        t.start()
        self._threads.append(t)

    def _guard(self, handler, c):
        try:
            if c is None:
                handler(c)
                return
            with c:
                handler(c)
        except BaseException as e:  # surfaced by Cluster.check()
            self.errors.append(e)

    def start(self) -> "Datanode":
        L = self.L
        self._serve(L.port(F.EC_WRITE_PORT), self._handle_write)
        self._serve(L.port(F.EC_READ_PORT), self._handle_read)
        if self.idx < L.k:
            self._serve(L.port(F.EC_WRITE_NEW_PORT), self._handle_write_new)
        else:
            if self.idx - L.k < L.ec_x:
                for eck in range(L.k):
                    self._serve(L.port(F.EC_WRITE_ECK_BASE_PORT + eck), self._handle_from_eck)
            for x in range(L.ec_x):
                self._serve(L.port(F.EC_WRITE_ECX_BASE_PORT + x), self._handle_coding_block)
        return self

    def stop(self, join: bool = True):
        self._stop.set()
        for s in self._socks:
            s.close()
        if join:
            self.join()

    def join(self):
        for t in self._threads:
            t.join(timeout=2)

    # -- -w / -r (eck_datanode_main.cpp:545-614, 286-314, 694-744)
    def _handle_write(self, c):
        md = self.L.unpack(_recv_exact(c, self.L.md_size))
        _send_int(c, 1)
        if md["block_size"] != -1:
            raise RuntimeError(f"handle_client_write: not a chunk (cur_eck {md['cur_eck']})")
        data = _recv_exact(c, md["chunk_size"])
        with self._io, open(self.path(md["dst_filename_datanode"]), "wb") as f:
            f.write(data)
        _send_int(c, 0)  # after the write, so a finished client call means the file is on disk

    def _handle_read(self, c):
        md = self.L.unpack(_recv_exact(c, self.L.md_size))
        with open(self.path(md["dst_filename_datanode"]), "rb") as f:
            data = f.read(md["chunk_size"])
        if len(data) != md["chunk_size"]:
            raise RuntimeError("handle_client_read: short chunk file")
        c.sendall(data)

    # -- block files + chunk_ok (eck_datanode_main.cpp:180-285)
    def _save_block(self, md: dict, data: bytes) -> None:
        off = F.block_offset(md["cur_block"], md["block_size"], md["remain_block_size"], md.get("net_block_size"))
        name = md["dst_filename_datanode"]
        p = self.path(name)
        with self._io:
            with open(p, "r+b" if os.path.exists(p) else "w+b") as f:
                f.seek(off)
                f.write(data)
            n = self._count.get(name, 0) + 1
            done = n == self.L.ec_n
            self._count[name] = 0 if done else n
        if done:  # chunk_ok to the client from the IO thread (:249-281)
            threading.Thread(target=self._guard, args=(self._chunk_ok, None), daemon=True).start()

    def _chunk_ok(self, _):
        with _connect(self.L.ip(-1), self.L.port(F.EC_WRITE_PORT), self.addr) as s:
            _send_int(s, 1)
            if _recv_int(s) == 0:
                raise RuntimeError("chunk_ok not acknowledged")

    # -- ECK: client blocks in, store + forward (eck_datanode_main.cpp:393-543, 315-391)
    def _handle_write_new(self, c):
        L = self.L
        ecx = [_connect(L.ip(L.k + i), L.port(F.EC_WRITE_ECK_BASE_PORT + self.idx), self.addr) for i in range(L.ec_x)]
        try:
            while True:
                raw = _recv_exact(c, L.md_size)
                md = L.unpack(raw)
                _send_int(c, 1)
                if not 0 <= md["cur_eck"] < L.k:
                    raise RuntimeError(f"handle_client_write_new: cur_eck {md['cur_eck']}")
                data = _recv_exact(c, md["block_size"])
                _send_int(c, 0)
                self._save_block(md, data)
                _send_metadata_and(ecx[md["cur_block"] % L.ec_x], raw, data)
                if md["cur_block"] == L.ec_n - 1:
                    break
        finally:
            for s in ecx:
                s.close()

    # -- ECX: ECK blocks in, in (block, eck) order; accumulate (ecx_datanode_main.cpp:1056-1146, 667-735)
    def _handle_from_eck(self, c):
        L = self.L
        while True:
            try:
                raw = _recv_exact(c, L.md_size)
            except ConnectionError:
                return
            md = L.unpack(raw)
            _send_int(c, 1)
            key = (md["cur_eck"], md["cur_block"])
            with self._gate:
                if not self._gate.wait_for(lambda: self._next == key, timeout=TIMEOUT_S):
                    raise RuntimeError(f"ECX {self.idx}: block {key} never became next ({self._next})")
                data = _recv_exact(c, md["block_size"])
                _send_int(c, 0)
                self._encode_block(md, data)
                eck, blk = key
                self._next = (eck + 1, blk) if eck + 1 < L.k else (
                    0, blk + L.ec_x if blk + L.ec_x < L.ec_n else self.idx - L.k)
                self._gate.notify_all()
            if md["cur_block"] >= L.ec_n - L.ec_x:  # this node's last block from this ECK (:1139-1142)
                return

    def _encode_block(self, md: dict, data: bytes) -> None:
        L, eck, size = self.L, md["cur_eck"], md["block_size"]
        if eck == 0:
            self._acc = self.coder.accumulator(L.m, size)
        block = np.frombuffer(data, np.uint8).copy()
        self._acc.add(block, [self.matrix[r * L.k + eck] for r in range(L.m)])
        if eck != L.k - 1:
            return
        x = self.idx - L.k
        for r in range(L.m):
            out = np.zeros(size, np.uint8)
            self._acc.read(r, out, size)
            cmd = dict(md)
            cmd["dst_filename_datanode"] = F.replace_filename_suffix(md["dst_filename_datanode"], L.k + r + 1)
            cmd["data"] = 0
            if r == x:
                self._save_block(cmd, out.tobytes())
            else:
                raw = L.pack(**cmd)
                with _connect(L.ip(L.k + r), L.port(F.EC_WRITE_ECX_BASE_PORT + x), self.addr) as s:
                    _send_metadata_and(s, raw, out.tobytes())
        self._acc = None

    # -- coding node: a coding block from an ECX node
    def _handle_coding_block(self, c):
        md = self.L.unpack(_recv_exact(c, self.L.md_size))
        _send_int(c, 1)
        data = _recv_exact(c, md["block_size"])
        _send_int(c, 0)
        self._save_block(md, data)


class Cluster:
    def __init__(self, root: str, coder: Coder, layout: Optional[Layout] = None, down: Sequence[int] = ()):
        self.L = layout or Layout()
        self.root, self.coder = root, coder
        self.matrix = coder.coding_matrix(self.L.k, self.L.m, self.L.w)
        self.nodes = {i: Datanode(self.L, i, root, coder, self.matrix)
                      for i in range(self.L.k + self.L.m) if i not in set(down)}

    def __enter__(self):
        for n in self.nodes.values():
            n.start()
        return self

    def __exit__(self, *exc):
        for n in self.nodes.values():
            n.stop(join=False)
        for n in self.nodes.values():
            n.join()
        return False

    def kill(self, idx: int) -> None:
        self.nodes.pop(idx).stop()

    def check(self) -> None:
        errs = [e for n in self.nodes.values() for e in n.errors]
        if errs:
            raise errs[0]

    def chunk_file(self, idx: int, name: str) -> str:
        return os.path.join(self.root, f"node{idx}", name)

    def client(self) -> "Client":
        return Client(self)


class Client:
    """The reference client's three commands (client_main.cpp:2202-2266)."""

    def __init__(self, cluster: Cluster):
        self.C, self.L = cluster, cluster.L
        self.base = os.path.join(cluster.root, "client")
        for d in (F.WRITE_PATH, F.READ_PATH, os.path.dirname(F.FILE_SIZE_PATH)):
            os.makedirs(os.path.join(self.base, d), exist_ok=True)

    def src_path(self, name: str) -> str:
        return os.path.join(self.base, F.WRITE_PATH, name)

    def _sidecar(self, dst: str) -> str:
        return os.path.join(self.base, F.FILE_SIZE_PATH + dst)

    def _buffers(self):
        L = self.L
        stripe = bytearray(L.k * L.chunk_size)
        data = [np.frombuffer(stripe, np.uint8, L.chunk_size, i * L.chunk_size) for i in range(L.k)]
        coding = [np.zeros(L.chunk_size, np.uint8) for _ in range(L.m)]
        return stripe, data, coding

    def _write_sidecar(self, dst: str, file_size: int) -> None:
        with open(self._sidecar(dst), "wb") as f:
            f.write(F.file_size_sidecar(file_size))

    # -w (client_main.cpp:1590-1918)
    def write(self, src: str, dst: str, test_n: int = 1, single_stripe_only: bool = True) -> int:
        L = self.L
        path = self.src_path(src)
        file_size = os.path.getsize(path)
        reading = F.stripe_count(file_size, L.k, L.chunk_size)
        if single_stripe_only and reading != 1:  # :1690-1695 ("For Test")
            return F.EC_ERROR
        stripe, data, coding = self._buffers()
        with open(path, "rb") as f:
            for cur in range(1, reading + 1):
                full = F.read_file_to_buffer(f, stripe)
                if single_stripe_only and full == 0:  # :1710-1715
                    return F.EC_ERROR
                name = F.stripe_filename(F.WRITE_PATH + dst, cur)
                for _ in range(test_n):
                    self.C.coder.encode(L.k, L.m, L.w, self.C.matrix, data, coding, L.chunk_size)
                    for i in range(L.k + L.m):  # send_chunks_datanodes_k / _m (:680-858), SEND_METHOD 1: serial
                        md = L.pack(chunk_size=L.chunk_size, block_size=-1,
                                    dst_filename_datanode=F.chunk_filename(name, i))
                        buf = data[i] if i < L.k else coding[i - L.k]
                        with _connect(L.ip(i), L.port(F.EC_WRITE_PORT), L.ip(-1)) as s:
                            _send_metadata_and(s, md, buf.tobytes())
        self._write_sidecar(dst, file_size)
        return F.EC_OK

    # -kw (client_main.cpp:1420-1588, 381-557)
    def write_eck(self, src: str, dst: str, test_n: int = 1) -> int:
        L = self.L
        path = self.src_path(src)
        file_size = os.path.getsize(path)
        if F.stripe_count(file_size, L.k, L.chunk_size) != 1:  # :1497-1502
            return F.EC_ERROR
        bs, rem = F.eck_block_sizes(L.chunk_size, L.w, L.ec_n)
        blocks = F.eck_blocks(L.chunk_size, L.w, L.ec_n)
        stripe, data, _ = self._buffers()
        with open(path, "rb") as f:
            F.read_file_to_buffer(f, stripe)  # -kw pads a short file (no io_flag check, :1516-1522)
        name = F.stripe_filename(F.WRITE_PATH + dst, 1)
        ok = _listen(L.ip(-1), L.port(F.EC_WRITE_PORT))
        ok.settimeout(TIMEOUT_S)
        try:
            for _ in range(test_n):
                socks = [_connect(L.ip(i), L.port(F.EC_WRITE_NEW_PORT), L.ip(-1)) for i in range(L.k)]
                try:
                    for j in range(L.ec_n):
                        for i in range(L.k):
                            off, size = blocks[j]
                            md = L.pack(sockfd=socks[i].fileno(), chunk_size=L.chunk_size, block_size=size,
                                        remain_block_size=rem, cur_block=j, cur_eck=i,
                                        dst_filename_datanode=F.chunk_filename(name, i), net_block_size=[bs] * L.ec_x)
                            _send_metadata_and(socks[i], md, data[i][off:off + size].tobytes())
                    for _ in range(L.k + L.m):  # chunk_ok from every node (:522-548)
                        c, _ = ok.accept()
                        with c:
                            c.settimeout(TIMEOUT_S)
                            _recv_int(c)
                            _send_int(c, 1)
                finally:
                    for s in socks:
                        s.close()
        finally:
            ok.close()
        self.C.check()
        self._write_sidecar(dst, file_size)
        return F.EC_OK

    # -r (client_main.cpp:1920-2195)
    def read(self, out: str, dst: str) -> int:
        L = self.L
        out_path = os.path.join(self.base, F.READ_PATH, out)
        with open(self._sidecar(dst), "rb") as f:
            file_size = F.parse_file_size_sidecar(f.read())
        remain_chunks, remain_size = F.read_tail(file_size, L.k, L.chunk_size)
        reading = F.stripe_count(file_size, L.k, L.chunk_size)
        _, data, coding = self._buffers()
        erasures = [-1] * (L.k + L.m)
        num_need_coding = 0
        with open(out_path, "wb") as fout:
            for cur in range(1, reading + 1):
                name = F.stripe_filename(F.WRITE_PATH + dst, cur)
                n_er = 0
                for i in range(L.k):  # recv_data_chunks_datanodes (:891-962)
                    if not self._fetch(i, name, data[i]):
                        erasures[n_er] = i
                        n_er += 1
                if cur == 1:  # :2074-2092
                    num_need_coding = sum(1 for i in range(L.k) if erasures[i] != -1)
                    if num_need_coding > L.m:
                        return F.EC_ERROR
                if num_need_coding:
                    tmp = num_need_coding  # recv_coding_chunks_datanodes (:964-1046): counts attempts, not successes
                    for i in range(L.k, L.k + L.m):
                        if tmp <= 0:
                            break
                        tmp -= 1
                        if not self._fetch(i, name, coding[i - L.k]):
                            erasures[n_er] = i
                            n_er += 1
                    if self.C.coder.decode(L.k, L.m, L.w, self.C.matrix, erasures, data, coding, L.chunk_size) != 0:
                        return F.EC_ERROR
                if cur != reading:
                    for i in range(L.k):
                        fout.write(data[i].tobytes())
                else:
                    fout.write(F.last_stripe_bytes(data, remain_chunks, remain_size))
        return F.EC_OK

    def _fetch(self, idx: int, name: str, into: np.ndarray) -> bool:
        L = self.L
        try:
            s = _connect(L.ip(idx), L.port(F.EC_READ_PORT), L.ip(-1))
        except OSError:
            return False  # a dead datanode becomes an erasure (:903-913)
        with s:
            s.sendall(L.pack(chunk_size=L.chunk_size, dst_filename_datanode=F.chunk_filename(name, idx)))
            into[:] = np.frombuffer(_recv_exact(s, L.chunk_size), np.uint8)
        return True
