"""Tuner, correlator, hw_stats and plotting helpers (CPU)."""
import csv
import json
import os

import numpy as np
import pytest

from accel_sim_framework_distributed_amd.job_launching import common, get_stats
from accel_sim_framework_distributed_amd.plotting import correlate, stats_plots
from accel_sim_framework_distributed_amd.tuner import tuner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UBENCH = os.path.join(ROOT, "profiles", "ubench_mi355x")


@pytest.mark.slow
def test_tuner_from_measured_mi355x_logs(native, tmp_path):
    opts, meas, dev = tuner.parse_stats([UBENCH])
    assert dev == "AMD_Instinct_MI355X"
    assert opts["-gpgpu_n_clusters"] == "256" and "-gpgpu_l1_latency" in opts
    assert float(meas["hbm_read_gbps"]) > 1000
    out, applied = tuner.tune([UBENCH], "MI355X", str(tmp_path))
    cfg = native.parse_config(["-config", os.path.join(out, "gpgpusim.config"), "-config",
                               os.path.join(out, "trace.config")])
    # the chain self-consistency takes the pipeline's own stages out of the
    # measured L1-hit pointer-chase latency (tuner._latency_self_consistency)
    assert cfg["n_sm"] == 256 and 0 < int(opts["-gpgpu_l1_latency"]) - cfg["l1_latency"] <= 16
    assert "TUNING.md" in os.listdir(out)
    # measured write policies (ub_cache_policy): L1 write-evict + lazy fetch
    # on read; the L2 probe reads a stored line back from memory but the L2
    # keeps store hits: write-back with byte-masked allocation ('L', the
    # counters show the L2 combining stores)
    assert applied["-gpgpu_cache:dl1"].split(",")[1].split(":")[1:4:2] == ["E", "L"]
    assert applied.get("-gpgpu_cache:dl2", "N:128:128:16,L:B:m:L:P").split(",")[1].split(":")[1:4:2] == ["B", "L"]


def test_tuner_rejects_unknown_flags(tmp_path):
    p = tmp_path / "x.log"
    p.write_text("-not_a_real_flag 3\n")
    with pytest.raises(ValueError):
        tuner.tune([str(p)], "QV100", str(tmp_path))


def test_tuner_search_space_resolves(native):
    from accel_sim_framework_distributed_amd.models import presets
    names = tuner.search_configs("QV100")
    assert len(names) == 16
    reg = common.Registry()
    for n in names:
        name, extra, base = reg.config(n)
        assert os.path.exists(base)
        for tok in n.split("-")[1:]:
            assert f"#{tok}\n" in extra
        args = list(presets.args_for("QV100"))
        for line in extra.splitlines():
            if line.startswith("-"):
                k, v = line.split(None, 1)
                args += [k, v]
        native.parse_config(args)  # every combination is a valid configuration


def _write_sim_csv(path, rows, cfg="MI355X"):
    # rows: {app/args: [cycles per kernel]}
    t = get_stats.StatTable()
    t.stats = [r"gpu_sim_cycle\s*=\s*(.*)"]
    for app, ks in rows.items():
        for i, c in enumerate(ks):
            t.set(app, f"k{i}--0", cfg, t.stats[0], str(c))
    open(path, "w").write(get_stats.render_csv(t))


def test_correlator_metrics_flat_hw(tmp_path):
    sim = {"a/x": [100, 200], "b/y": [300], "c/z": [1000]}
    hw_cycles = {"a/x": [110, 190], "b/y": [250], "c/z": [1000]}
    _write_sim_csv(tmp_path / "s.csv", sim)
    with open(tmp_path / "hw.csv", "w") as f:
        f.write("app,args,kernel,instance,duration_ns\n")
        for app, ks in hw_cycles.items():
            a, g = app.split("/")
            for i, c in enumerate(ks):
                for rep in range(3):
                    f.write(f"{a},{g},k{i},{i},{c * 1000 / 2000.0}\n")  # ns at 2000 MHz
    hw = correlate.load_hw_flat(str(tmp_path / "hw.csv"))
    res = correlate.correlate(str(tmp_path / "s.csv"), hw, 2000.0)
    m = res["Cycles"]["configs"]["MI355X"]["app_metrics"]
    # per app: a 300 vs 300 (0%), b 300 vs 250 (20%), c 0%  -> MAE 6.67%
    assert m["n"] == 3 and m["mae"] == pytest.approx(20 / 3, rel=1e-6)
    files = correlate.write_outputs(res, str(tmp_path / "out"))
    summ = json.load(open([f for f in files if f.endswith(".json")][0]))
    assert summ["Cycles"]["MI355X"]["app"]["n"] == 3
    assert any(f.endswith(".html") and "<svg" in open(f).read() for f in files)


def test_correlator_rocprof_loader(tmp_path):
    d = tmp_path / "hw" / "vectoradd" / "NO_ARGS"
    for r in range(3):
        rd = d / f"run_{r}" / "host" / "123"
        rd.mkdir(parents=True)
        with open(rd / "run_kernel_trace.csv", "w") as f:
            w = csv.writer(f)
            w.writerow(["Kind", "Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
            w.writerow(["KERNEL_DISPATCH", 2, "void k2(int*)", 5000, 5000 + 800 + r])
            w.writerow(["KERNEL_DISPATCH", 1, "void k1(int*) [clone .kd]", 1000, 1000 + 400 + r])
    hw = correlate.load_hw_rocprof(str(tmp_path / "hw"), burn=1)
    ks = hw["vectoradd/NO_ARGS"]
    assert len(ks) == 2 and ks[0]["duration_ns"] == [401.0, 402.0] and ks[1]["name"] == ["void k2"]


def test_run_hw_dry_run(capsys):
    from accel_sim_framework_distributed_amd.hw_stats import run_hw
    assert run_hw.main(["-B", "asim_hip_apps", "-R", "2", "-n", "-o", "/tmp/x"]) == 0
    out = capsys.readouterr().out
    assert out.count("rocprofv3 --kernel-trace") == 20 and "bin/apps/vectoradd 262144" in out  # 10 app inputs x 2 runs


def test_stats_merge_and_plot(tmp_path):
    _write_sim_csv(tmp_path / "a.csv", {"a/x": [1, 2]}, "C1")
    _write_sim_csv(tmp_path / "b.csv", {"a/x": [3, 4]}, "C2")
    merged = stats_plots.merge([str(tmp_path / "a.csv"), str(tmp_path / "b.csv")])
    blocks = get_stats.parse_csv_blocks(merged)
    row = blocks[r"gpu_sim_cycle\s*=\s*(.*)"]["a/x--k0--0"]
    assert row == {"C1": "1", "C2": "3"}
    (tmp_path / "m.csv").write_text(merged)
    files = stats_plots.plot(str(tmp_path / "m.csv"), str(tmp_path / "html"))
    assert files and "<svg" in open(files[0]).read()


def test_trace_tools_cli(native, tmp_path, capsys):
    from accel_sim_framework_distributed_amd.tracegen import cli
    assert cli.main(["generate", "-o", str(tmp_path), "-a", "bfs-rodinia-2.0-ft"]) == 0
    kl = [os.path.join(r, f) for r, _, fs in os.walk(tmp_path) for f in fs if f == "kernelslist.g"][0]
    d = os.path.dirname(kl)
    assert cli.main(["info", d]) == 0
    assert cli.main(["occupancy", d]) == 0
    out = capsys.readouterr().out
    assert "CTAs/SM, limited by" in out and "#thread insts" in out
    bbv_path = str(tmp_path / "bbv.json")
    assert cli.main(["bbv", d, "-o", bbv_path]) == 0
    bbv = json.load(open(bbv_path))
    assert len(bbv) >= 2 and all(sum(v.values()) > 0 for v in bbv.values())
    # every thread instruction lands in exactly one basic block
    info = {os.path.basename(p): native.kernel_info(p)["thread_insts"] for p in cli.kernel_files(d)}
    for k, v in bbv.items():
        assert sum(v.values()) == info[k]
    before = {k: native.kernel_info(p)["warp_insts"] for k, p in zip(info, cli.kernel_files(d))}
    assert cli.main(["convert", d, "--to", "text"]) == 0
    assert cli.main(["convert", d, "--to", "binary"]) == 0
    after = {os.path.basename(p): native.kernel_info(p)["warp_insts"] for p in cli.kernel_files(d)}
    assert before == after


def test_ubench_output_parser():
    from accel_sim_framework_distributed_amd.ops import ubench
    log = open(os.path.join(UBENCH, "ub_cache_lat.log")).read()
    r = ubench.parse(log)
    assert r["options"]["-gpgpu_l1_latency"] and float(r["measurements"]["xcd_l2_hit_latency"]) > 0


def test_correlator_stat_breadth_matches_simulator_output(tmp_path):
    """>= 15 CorrelStats, and every simulator regex they use is in the stats
    yml and matches a line of a real simulator run (per kernel)."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    assert len(correlate.CORREL_STATS) >= 15
    spec = get_stats.load_stats_yml("")
    listed = set(spec["collect_aggregate"] + spec["collect_abs"] + spec["collect_rates"])
    kl = rodinia.write_app(str(tmp_path / "bp"), rodinia.backprop(1024))
    out = sim.simulate(kl, "QV100", engine="cpu").output
    per, order = get_stats.parse_output(out, spec, per_kernel=True, kernel_instance=True)
    assert len(order) == 2
    for st in correlate.CORREL_STATS:
        for rx in (st.sim_stats or (st.sim_stat,)):
            assert rx in listed, rx
            assert all(rx in per[k] for k in order), rx
    # cumulative counters are differenced back to per-kernel values
    l2r = r"\s+L2_cache_stats_breakdown\[GLOBAL_ACC_R\]\[TOTAL_ACCESS\]\s*=\s*(.*)"
    vals = [int(per[k][l2r]) for k in order]
    raw = [int(l.split("=")[1]) for l in out.splitlines() if "L2_cache_stats_breakdown[GLOBAL_ACC_R][TOTAL_ACCESS]" in l]
    assert raw[1] >= raw[0] and vals == [raw[0], raw[1] - raw[0]]


def test_correlator_counter_passes_and_derived_stats(tmp_path):
    """Counter-pass directories (ctr<g>_<i>) merge into the kernel records and
    derived stats (IPC, hit rates) are evaluated kernel by kernel."""
    S = correlate
    t = get_stats.StatTable()
    stats = {S.S_CYC: [1000, 2000], S.S_WINSN: [500, 3000],
             # MI355X semantics: every write is an L2 hit, read misses and the
             # reads merged into them are the misses
             S.S_L2 % ("GLOBAL_ACC_R", "HIT"): [60, 10], S.S_L2 % ("GLOBAL_ACC_W", "TOTAL_ACCESS"): [20, 10],
             S.S_L2 % ("GLOBAL_ACC_R", "MISS"): [15, 70], S.S_L2 % ("GLOBAL_ACC_R", "MSHR_HIT"): [5, 10]}
    t.stats = list(stats)
    for s, ks in stats.items():
        for i, v in enumerate(ks):
            t.set("app/x", f"k{i}--0", "MI355X", s, str(v))
    (tmp_path / "s.csv").write_text(get_stats.render_csv(t))
    d = tmp_path / "hw" / "app" / "x"
    for r in range(2):
        rd = d / f"run_{r}"
        rd.mkdir(parents=True)
        with open(rd / "k_kernel_trace.csv", "w") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
            w.writerow([1, "k0", 0, 500])      # 1000 cycles at 2000 MHz
            w.writerow([2, "k1", 1000, 2000])  # 2000 cycles
    cd = d / "ctr0_0"
    cd.mkdir()
    with open(cd / "c_counter_collection.csv", "w") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writerow([7, "__amd_rocclr_fillBuffer", "TCC_HIT", 999])
        for disp, hit, miss in ((8, 40, 10), (9, 30, 30)):
            w.writerow([disp, "k", "TCC_HIT", hit / 2])   # two dimension instances
            w.writerow([disp, "k", "TCC_HIT", hit / 2])
            w.writerow([disp, "k", "TCC_MISS", miss])
            w.writerow([disp, "k", "SQ_INSTS_VALU", 250 if disp == 8 else 1000])
    hw = S.load_hw_rocprof(str(tmp_path / "hw"), burn=0)
    k = hw["app/x"]
    assert k[0]["TCC_HIT_sum"] == [40.0] and k[1]["TCC_MISS_sum"] == [30.0]
    res = S.correlate(str(tmp_path / "s.csv"), hw, 2000.0)
    hr = res["L2 hit rate"]["configs"]["MI355X"]
    # per kernel: sim 0.8 / 0.2, hw 0.8 / 0.5 -> per-app means 0.5 vs 0.65
    (hwv, simv, _), = hr["apps"]
    assert simv == pytest.approx(0.5) and hwv == pytest.approx(0.65)
    assert res["Cycles"]["configs"]["MI355X"]["app_metrics"]["mae"] == pytest.approx(0.0)
