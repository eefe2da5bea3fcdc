"""Every evidence file under profiles/ is named in profiles/INDEX.md (what it
is and which command made it), and every profile the bench line cites
exists."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def test_every_profile_is_indexed():
    index = open(os.path.join(PROF, "INDEX.md")).read()
    missing = [f for f in sorted(os.listdir(PROF)) if f != "INDEX.md" and f not in index]
    assert not missing, missing


def test_bench_traffic_record_is_committed():
    # bench.py reads roofline.traffic from the committed PMC record of the kernel build it loads
    summary = json.load(open(os.path.join(PROF, "r05_rocprof_summary.json")))
    assert summary["kernel_build_id"] and summary["kernels"]["encode"]["traffic_over_algorithmic"] < 1.01
    for f in ("pmc_encode.json", "pmc_decode.json", "r05_kernel_stats.csv", "r05_bench.json"):
        assert os.path.exists(os.path.join(PROF, f)), f
    # the committed PMC records are for the w = 8 kernel build of the closing profile pass
    for f in ("pmc_encode.json", "pmc_decode.json"):
        assert json.load(open(os.path.join(PROF, f)))["kernel_build_id"] == summary["kernel_build_id"]


def _skew_table():
    """{size: skew} from csrc/shard_stride.hpp's kSkewTable."""
    import re
    src = open(os.path.join(ROOT, "erasure_coding_test_amd", "csrc", "shard_stride.hpp")).read()
    body = src[src.index("kSkewTable[] = {"):src.index("};", src.index("kSkewTable[] = {"))]
    def ev(e):  # "12 << 10" -> 12288
        parts = [int(x) for x in e.split("<<")]
        return parts[0] << sum(parts[1:])
    table = {ev(a): ev(b) for a, b in re.findall(r"\{([\d <]+),\s*([\d <]+)\}", body)}
    no_skew = ev(re.search(r"kNoSkewUpTo = ([\d <]+);", src).group(1))
    return table, no_skew


def test_stride_statements_agree_with_the_table():
    """the bench's stride comment, the C header and the
    DESIGN §4 table state the skews the library actually uses."""
    import re
    t, no_skew = _skew_table()
    mib, kib = 1 << 20, 1 << 10
    assert t[4 * mib] == 6 * kib and t[16 * mib] == 8 * kib and t[1 * mib] == 0
    assert no_skew == 256 * kib and t[256 * kib] == 0 and t[512 * kib] == 0  # round 5: small shards take no skew
    bench_src = open(os.path.join(ROOT, "bench.py")).read()
    assert "6 KiB at 4 MiB, 8 KiB at 16 MiB" in bench_src and "S + 10 KiB" not in bench_src
    hdr = open(os.path.join(ROOT, "include", "ecgpu.h")).read()
    assert "6 KiB at 4 MiB, 8 KiB at 16 MiB, none at 1 MiB" in hdr
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    sizes = re.search(r"\| shard size \(±1/16\) \|(.*)\|", design).group(1).split("|")
    skews = re.search(r"\| skew \(KiB\) \|(.*)\|", design).group(1).split("|")
    got = {}
    for sz, sk in zip(sizes, skews):
        sz, sk = sz.strip(), sk.strip().strip("*")
        if sz == "other":
            continue
        if sz.startswith("≤"):  # the no-skew rule's column: every table class up to it
            sz = sz[1:].strip()
            assert int(sz.split()[0]) * kib == no_skew and sk == "0", (sz, sk)
            got.update({n: 0 for n in t if n <= no_skew})
            continue
        n = int(sz.split()[0]) * (kib if sz.endswith("K") else mib)
        got[n] = int(sk) * kib
    assert got == t
