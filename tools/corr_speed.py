#!/usr/bin/env python3
"""Speed and accuracy of one correlation run, from the same simulations:
total simulated thread instructions of every job (the last gpu_tot_sim_insn
of each job's output under <simrun>) over the run's wall time, next to the
cycle MAE the correlator computed from those jobs (<correl>/mi355x-summary.json).
usage: corr_speed.py <simrun_dir> <correl_dir> <wall_s> <label>"""
import glob
import json
import os
import re
import sys


def main():
    simrun, correl, wall, label = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    insn = 0
    jobs = 0
    for f in glob.glob(os.path.join(simrun, "*", "*", "*", "*.o*")):
        v = re.findall(r"^gpu_tot_sim_insn = (\d+)", open(f, errors="replace").read(), re.M)
        if v:
            insn += int(v[-1])
            jobs += 1
    d = json.load(open(os.path.join(correl, "mi355x-summary.json")))
    cyc = d["Cycles"][list(d["Cycles"])[0]]
    out = {"label": label, "jobs": jobs, "sim_insn": insn, "wall_s": round(wall, 2),
           "kips": round(insn / wall / 1e3, 1), "config": list(d["Cycles"])[0],
           "cycle_mae_all_apps": round(cyc["app_incl_noisy"]["mae"], 2), "apps": cyc["app_incl_noisy"]["n"],
           "cycle_mae_stable_apps": round(cyc["app"]["mae"], 2), "pearson": round(cyc["app_incl_noisy"]["correl"], 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
