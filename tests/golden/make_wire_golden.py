"""Generate tests/golden/wire.json from the REFERENCE's own header.

Runs only where /root/reference exists.  Compiles a small C program (written
to a temp dir, never committed) that includes the reference's
include/ych_ec_test.h unchanged and prints what gcc makes of ``metadata_t``:
its size, every field offset, and the raw byte image of sample structs built
the way the reference's senders build them (memset of the name, sprintf of the
chunk file name, the file-size sidecar buffer).  Only that data is stored.

    python tests/golden/make_wire_golden.py
"""
from __future__ import annotations

import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = "/root/reference/include/ych_ec_test.h"

PROGRAM = r"""
#include <stdio.h>
#include <stddef.h>
#include <string.h>
#include "%s"
static void hex(const void *p, size_t n) {
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; i++) printf("%%02x", b[i]);
}
int main(void) {
    printf("{\"sizeof\": %%zu, \"offsets\": {", sizeof(metadata_t));
    printf("\"sockfd\": %%zu, \"chunk_size\": %%zu, \"block_size\": %%zu, \"remain_block_size\": %%zu, ",
           offsetof(metadata_t, sockfd), offsetof(metadata_t, chunk_size), offsetof(metadata_t, block_size),
           offsetof(metadata_t, remain_block_size));
    printf("\"cur_block\": %%zu, \"cur_eck\": %%zu, \"data\": %%zu, \"dst_filename_datanode\": %%zu, ",
           offsetof(metadata_t, cur_block), offsetof(metadata_t, cur_eck), offsetof(metadata_t, data),
           offsetof(metadata_t, dst_filename_datanode));
    printf("\"error_flag\": %%zu, \"net_block_size\": %%zu}, ", offsetof(metadata_t, error_flag),
           offsetof(metadata_t, net_block_size));
    printf("\"EC_X\": %%d, \"EC_K\": %%d, \"EC_M\": %%d, \"EC_N\": %%d, \"EC_W\": %%d, \"MAX_PATH_LEN\": %%d, ",
           EC_X, EC_K, EC_M, EC_N, EC_W, MAX_PATH_LEN);
    /* a whole-chunk write (client_main.cpp:617-635) and an ECK block (:420-436) */
    metadata_t a, b;
    memset(&a, 0, sizeof a); memset(&b, 0, sizeof b);
    a.sockfd = 7; a.chunk_size = 1048576; a.block_size = -1; a.error_flag = EC_OK;
    a.data = (char *)0x7f00deadbeef0ull;
    sprintf(a.dst_filename_datanode, "%%s_%%d", "/data/test_file/write/dst1", 5);
    b.sockfd = 9; b.chunk_size = 1048576; b.block_size = 349525; b.remain_block_size = 1;
    b.cur_block = 2; b.cur_eck = 1; b.error_flag = EC_ERROR;
    sprintf(b.dst_filename_datanode, "%%s_%%d", "x/test_file/write/f1", 2);
    for (int i = 0; i < EC_X; i++) b.net_block_size[i] = 349525 + i;
    printf("\"chunk_image\": \""); hex(&a, sizeof a);
    printf("\", \"block_image\": \""); hex(&b, sizeof b);
    /* file-size sidecar (client_main.cpp:1886-1889) */
    char fsb[MAX_PATH_LEN] = {0};
    sprintf(fsb, "%%d", 3145728);
    printf("\", \"sidecar_3145728\": \""); hex(fsb, sizeof fsb);
    printf("\"}\n");
    return 0;
}
"""


def main():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "wire.c"), os.path.join(d, "wire")
        with open(src, "w") as f:
            f.write(PROGRAM % HEADER)
        subprocess.run(["gcc", "-O0", "-o", exe, src], check=True)
        out = json.loads(subprocess.run([exe], check=True, capture_output=True, text=True).stdout)
    out["generator"] = "tests/golden/make_wire_golden.py"
    out["source"] = "gcc on the reference's include/ych_ec_test.h (default build)"
    with open(os.path.join(HERE, "wire.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print("wrote", os.path.join(HERE, "wire.json"))


if __name__ == "__main__":
    main()
