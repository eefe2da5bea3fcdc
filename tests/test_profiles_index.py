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
    name, summary = _latest_rocprof_summary()
    tag = name[:3]
    assert summary["kernel_build_id"] and summary["kernels"]["encode"]["traffic_over_algorithmic"] < 1.01
    for f in ("pmc_encode.json", "pmc_decode.json", f"{tag}_kernel_stats.csv"):
        assert os.path.exists(os.path.join(PROF, f)), f
    # the committed PMC records are for the w = 8 kernel build of the closing profile pass
    for f in ("pmc_encode.json", "pmc_decode.json"):
        assert json.load(open(os.path.join(PROF, f)))["kernel_build_id"] == summary["kernel_build_id"]


def _latest_rocprof_summary():
    import re
    names = sorted(f for f in os.listdir(PROF) if re.fullmatch(r"r\d\d_rocprof_summary\.json", f))
    return names[-1], json.load(open(os.path.join(PROF, names[-1])))


def _ranges(cell):
    """'0.889–0.898 ms' -> [(0.889, 0.898)]; 'a–b / c' -> [(a, b), (c, c)]."""
    import re
    out = []
    for part in cell.replace("ms", "").split("/"):
        nums = [float(x) for x in re.findall(r"\d+\.\d+", part)]
        assert nums, cell
        out.append((min(nums), max(nums)))
    return out


def test_kernel_bound_table_brackets_the_latest_rocprof_medians():
    """DESIGN §5's bound table (time and fraction of the
    8 TB/s spec per BASELINE launch) must bracket the medians of the latest
    committed rocprof summary, so a stale row fails here."""
    name, summary = _latest_rocprof_summary()
    k = summary["kernels"]
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    section = design[design.index("**What bounds each kernel**"):design.index("### 5.1")]
    rows = {}
    for line in section.splitlines():
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if len(cells) == 5 and cells[0].startswith("`gf_apply<"):
            rows[cells[0]] = cells
    want = {  # table row -> summary kernels, in the row's "a / b" order
        "`gf_apply<10,4,3>`": ["encode"],
        "`gf_apply<10,1,4>`": ["decode"],
        "`gf_apply<10,1,1>`": ["C3_decode_parity"],
        "`gf_apply<10,4,0>`": ["C4_decode_0123"],
        "`gf_apply<6,3,3>` / `<12,4,3>`": ["C2_encode", "C5_encode"],
    }
    tol = 0.0015  # the table rounds to three decimals
    for row, keys in want.items():
        assert row in rows, (row, sorted(rows))
        _, _, t_cell, f_cell, _ = rows[row]
        times, fracs = _ranges(t_cell), _ranges(f_cell)
        assert len(times) == len(fracs) == len(keys), (row, t_cell, f_cell)
        for key, (t_lo, t_hi), (f_lo, f_hi) in zip(keys, times, fracs):
            med_ns = k[key]["median_duration_ns"]
            frac = k[key]["algorithmic_bytes_per_launch"] / med_ns / 8000.0
            assert t_lo - tol <= med_ns / 1e6 <= t_hi + tol, (name, row, key, med_ns, t_cell)
            assert f_lo - tol <= frac <= f_hi + tol, (name, row, key, round(frac, 4), f_cell)


def test_design_test_count_matches_the_latest_gpu_record():
    """the `-m gpu` test count DESIGN §3 states is the
    latest committed GPU-suite record's."""
    import re
    recs = sorted(f for f in os.listdir(PROF) if re.fullmatch(r"r\d\d_gputest\.txt", f))
    if not recs:
        return
    passed = re.findall(r"(\d+) passed", open(os.path.join(PROF, recs[-1])).read())
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    stated = re.search(r"`-m gpu`, (\d+) tests", design).group(1)
    assert passed and stated == passed[-1], (recs[-1], passed, stated)


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
