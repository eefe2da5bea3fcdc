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
    summary = json.load(open(os.path.join(PROF, "r04_rocprof_summary.json")))
    assert summary["kernel_build_id"] and summary["kernels"]["encode"]["traffic_over_algorithmic"] < 1.01
    for f in ("pmc_encode.json", "pmc_decode.json", "r04_kernel_stats.csv", "r04_bench.json"):
        assert os.path.exists(os.path.join(PROF, f)), f
