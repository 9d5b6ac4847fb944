"""merge-stats (reference util/plotting/merge-stats.py) and the AccelWattch power
CSV collector (reference util/accelwattch/gen_sim_power_csv.py)."""
import csv
import os
import subprocess
import sys

from accel_sim_framework_distributed_amd.job_launching.get_stats import StatTable, parse_csv_blocks, render_csv
from accel_sim_framework_distributed_amd.plotting import merge_stats
from accel_sim_framework_distributed_amd.power import collect

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table(cfg, build, cycles):
    t = StatTable()
    t.stats = ["Accel-Sim-build", "gpu_tot_sim_cycle\\s*=\\s*(.*)"]
    for i, (app, c) in enumerate(cycles.items()):
        t.set(app, "kern", cfg, "gpu_tot_sim_cycle\\s*=\\s*(.*)", str(c))
        t.set(app, "kern", cfg, "Accel-Sim-build", f"Accel-Sim [build {build}]")
    return render_csv(t)


def test_merge_stats_tags_builds_and_keeps_common_rows(tmp_path):
    a = _table("QV100-SASS", "abcdef1234", {"bfs/args": 100, "nw/args": 200})
    b = _table("QV100-SASS", "0123456789", {"bfs/args": 110, "lud/args": 50})
    merged = merge_stats.merge([("a.csv", a), ("b.csv", b)])
    blocks = parse_csv_blocks(render_csv(merged))
    rows = blocks["gpu_tot_sim_cycle\\s*=\\s*(.*)"]
    assert set(rows) == {"bfs/args--kern"}  # only rows present in every file
    assert rows["bfs/args--kern"] == {"QV100-SASS-accel-abcdef1": "100", "QV100-SASS-accel-0123456": "110"}
    # same build twice: the second copy is filtered out
    merged2 = merge_stats.merge([("a.csv", a), ("a2.csv", a)])
    assert len(merged2.configs) == 1


def test_merge_stats_cli(tmp_path):
    pa, pb = tmp_path / "a.csv", tmp_path / "b.csv"
    pa.write_text(_table("X", "1111111aaa", {"app/a": 1}))
    pb.write_text(_table("Y", "2222222bbb", {"app/a": 2}))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "util", "plotting", "merge-stats.py"), "-c",
                          f"{pa},{pb}"], capture_output=True, text=True, check=True).stdout
    assert "X-accel-1111111" in out and "Y-accel-2222222" in out


def test_power_csv_from_simulated_reports(native, tmp_path):
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.power import xmlcfg
    xml = str(tmp_path / "aw.xml")
    xmlcfg.write_xml(xml, xmlcfg.default_params("QV100"))
    reports = tmp_path / "accelwattch_power_reports" / "qv100_sass_sim"
    reports.mkdir(parents=True)
    for app, kernels in (("backprop", rodinia.backprop(1024)), ("vadd", [rodinia.vectoradd(20000)])):
        d = tmp_path / app
        d.mkdir()
        kl = rodinia.write_app(str(d / "traces"), kernels)
        extra = {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml}
        cwd = os.getcwd()
        os.chdir(d)
        try:
            s = native.Simulator(presets.args_for("QV100", extra) + ["-trace", kl], False)
            assert s.run() == 0
        finally:
            os.chdir(cwd)
        os.replace(d / "accelwattch_power_report.log", reports / f"{app}.log")
    out = tmp_path / "res"
    assert collect.main([str(tmp_path / "accelwattch_power_reports"), "all", "-o", str(out)]) == 0
    rows = list(csv.reader(open(out / "accelwattch_qv100_sass_sim.csv")))
    hdr, body = rows[0], {r[0]: r[1:] for r in rows[1:]}
    assert set(body) == {"backprop_k1", "backprop_k2", "vadd_k1"}
    assert "MCP" not in hdr and "NOCP" not in hdr and "DRAMP" in hdr  # SASS family drops, DRAM absorbs MC
    p = dict(zip(hdr[1:], map(float, body["vadd_k1"])))
    assert p["kernel_avg_power"] > 0 and p["STATICP"] >= 0
