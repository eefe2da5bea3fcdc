"""Why is the C3 encode slower inside bench.py's step than in tools/encode_lab?

Same process, same slab (E.alloc_stripes, the bench's layout), interleaved
rounds of:
  enc_only   20 back-to-back encode launches (the lab's pattern)
  step       20 x (encode, decode{0}) -- the bench's timed step
  step_dec1  20 x (encode, decode{1}) -- the decode rebuilding a shard the next
             encode does not read first
Each launch timed with HIP events on the launch stream; medians in us.
Also prints the slab base alignment.

  python tools/probe_step.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import erasure_coding_test_amd as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--stripes", type=int, default=96)
    ap.add_argument("--data", choices=["random", "same", "zero"], default="random",
                    help="shard contents: independent random bytes (the bench), one random shard copied "
                         "everywhere (tools/encode_lab.hip), or zeros")
    args = ap.parse_args()
    k, m, S, B = 10, 4, 4 << 20, args.stripes
    dev = torch.device("cuda", 0)
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab, shards = E.alloc_stripes(B, k, m, S, dev)
    if args.data == "random":
        slab.random_(0, 256)
    elif args.data == "same":
        one = torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev)
        for st in shards:
            for sh in st:
                sh.copy_(one)
    else:
        slab.zero_()
    enc = E.encode_plan(k, m, M, 0).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
    dec0 = E.DecodePlan(k, m, M, [0], 0, 0).bind_stripes(shards, S)
    dec1 = E.DecodePlan(k, m, M, [1], 0, 0).bind_stripes(shards, S)
    stream = torch.cuda.current_stream(dev)
    n = 20
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n + 1)]
    for e in evs:
        e.record(stream)
    torch.cuda.synchronize()

    def run(kind):
        for _ in range(3):
            enc.launch(stream.cuda_stream)
        evs[0].record(stream)
        for i in range(n):
            enc.launch(stream.cuda_stream)
            evs[2 * i + 1].record(stream)
            if kind == "step":
                dec0.launch(stream.cuda_stream)
            elif kind == "step_dec1":
                dec1.launch(stream.cuda_stream)
            evs[2 * i + 2].record(stream)
        torch.cuda.synchronize()
        e_ms = [evs[2 * i].elapsed_time(evs[2 * i + 1]) if i == 0 or kind == "enc_only"
                else evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(n)]
        if kind == "enc_only":  # consecutive encodes: launch i spans event 2i .. 2i+1, then an empty gap
            e_ms = [evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(n)]
        d_ms = [evs[2 * i + 1].elapsed_time(evs[2 * i + 2]) for i in range(n)] if kind != "enc_only" else []
        return statistics.median(e_ms) * 1e3, (statistics.median(d_ms) * 1e3 if d_ms else None)

    res = {"enc_only": [], "step": [], "step_dec1": []}
    for _ in range(args.rounds):
        for kind in res:
            res[kind].append(run(kind))
    out = {"data": args.data, "slab_base_mod_2MiB": slab.data_ptr() % (2 << 20), "slab_base_mod_64KiB": slab.data_ptr() % (64 << 10),
           "stride": int(slab.stride(1))}
    for kind, v in res.items():
        out[kind] = {"encode_us": [round(a, 1) for a, _ in v],
                     "decode_us": [round(b, 1) for _, b in v] if v[0][1] is not None else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
