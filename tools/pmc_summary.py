#!/usr/bin/env python3
"""Sum rocprofv3 PMC counters of the engine kernel (rocpd SQLite database)
and print per-wave ratios.  usage: pmc_summary.py <db> [kernel-substring]"""
import json
import sqlite3
import sys


def main():
    db = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "engine_kernel"
    c = sqlite3.connect(db)
    tot = {}
    meta = None
    for name, cnt, val, vg, ag, sg, sc, lds in c.execute(
            "select kernel_name, counter_name, value, vgpr_count, accum_vgpr_count, sgpr_count, scratch_size, "
            "lds_block_size from counters_collection"):
        if pat not in name:
            continue
        tot[cnt] = tot.get(cnt, 0.0) + float(val)
        meta = dict(vgpr=vg, agpr=ag, sgpr=sg, scratch=sc, lds=lds)
    out = dict(kernel_pattern=pat, counters=tot, kernel_resources=meta)
    w = tot.get("SQ_WAVE_CYCLES", 0)
    if w:
        out["share_of_wave_cycles"] = {k: round(tot[k] / w, 4) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
                                       if k in tot}
    ins = sum(tot.get(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"))
    if ins and w:
        out["wave_cycles_per_instruction(x4 quad)"] = round(4 * w / ins, 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
