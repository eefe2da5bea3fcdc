"""LDS model behind closing the w = 32 byte-table redesign (VERDICT r4 next #6,
DESIGN.md §10).

The w = 32 kernels are LDS-array-bound (72 % busy): per source dword 8 nibble
lookups, each one ds_read_b128 of a 16-entry x 16-B table (all R <= 4 rows'
32-bit products).  The proposed redesign looks bytes up instead: 4 lookups
per dword in 256-entry tables (16 B entries for R = 4, 8 B for R <= 2).
Half the lookups -- but LDS time is lookups x conflict degree.  LDS is 64
banks x 4 B (256 B per clock, MI355X_MICROARCH.md); a ds_read_b128 serves 16
lanes per pass, a ds_read_b64 32.  A pass costs the largest number of
DISTINCT entries that fall into one bank group (same-address lanes
broadcast).  A 16-entry x 16-B table spans each bank group exactly once, so
its lookups never conflict; a 256-entry table maps 16 (or 8) entries onto
each group, and random bytes collide.

    python tools/lds_conflict_model.py > profiles/r05_w32_byte_table_model.json
"""
import json

import numpy as np


def pass_cycles(lanes, entries, entry_bytes, trials=20000, seed=0):
    rng = np.random.default_rng(seed)
    groups = 256 // entry_bytes
    tot = 0
    for _ in range(trials):
        u = np.unique(rng.integers(0, entries, lanes))
        tot += np.bincount(u % groups, minlength=groups).max()
    return tot / trials


def main():
    nib128 = pass_cycles(16, 16, 16)
    byte128 = pass_cycles(16, 256, 16)
    nib64 = pass_cycles(32, 16, 8)
    byte64 = pass_cycles(32, 256, 8)
    cur = 8 * nib128  # nibble form, R = 3..4: 8 ds_read_b128 per source dword
    out = {
        "model": "LDS pass cycles per source dword = lookups x mean conflict degree (random bytes)",
        "conflict_degree": {"nibble_b128": nib128, "byte_b128": round(byte128, 3), "nibble_b64": nib64,
                            "byte_b64": round(byte64, 3)},
        "R4": {"nibble_form_units": cur, "byte_form_units": round(4 * byte128, 2),
               "byte_over_nibble": round(4 * byte128 / cur, 3)},
        "R2": {"nibble_form_units": 8 * nib64, "byte_form_units": round(4 * byte64, 2),
               "byte_over_nibble": round(4 * byte64 / (8 * nib64), 3)},
        "tables_per_workgroup_KiB": {"RS(10,4) w=32 byte form, 9 looked-up sources x 4 positions x 256 x 16 B": 144,
                                     "LDS per CU": 160},
        "verdict": "the byte-indexed form needs MORE LDS array time than the nibble form (x1.46 at R = 4, x1.58 at "
                   "R <= 2) and leaves one workgroup per CU: predicted slower, not >= 10 % faster; not built",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
