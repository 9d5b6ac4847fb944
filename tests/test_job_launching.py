"""Job-launching layer: run_simulations -> procman -> monitor_func_test/job_status -> get_stats
(reference util/job_launching/*, exercised the way its CI does: launch a suite
locally, wait with monitor_func_test, collect stats)."""
import os
import subprocess
import sys
import textwrap

import pytest

from accel_sim_framework_distributed_amd.job_launching import common, get_stats, procman


def test_argfoldername_matches_reference_rules():
    assert common.argfoldername(None) == "NO_ARGS"
    assert common.argfoldername("4096 ./data/result-4096.txt") == "4096___data_result_4096_txt"
    long = "x" * 300
    assert common.argfoldername(long).startswith("hashed_args_")


def test_registry_suites_and_configs():
    reg = common.Registry()
    r = reg.benchmarks(["rodinia_2.0-ft"])
    assert len(r) == 10
    from accel_sim_framework_distributed_amd.tracegen.rodinia import SUITE
    for _, _, app, args in r:
        assert common.argfoldername(args[0]["args"]) == SUITE[app][0]
    name, extra, base = reg.config("QV100-GPU-L1OFF")
    assert "-sim_engine gpu" in extra and "-gpgpu_gmem_skip_L1D 1" in extra
    assert os.path.exists(base)
    with pytest.raises(KeyError):
        reg.config("QV100-NOPE")


def test_procman_selftest():
    assert procman.self_test() == 0


def test_stats_parsing_per_kernel():
    out = textwrap.dedent("""\
        Accel-Sim-AMD [MI355X-native trace-driven simulator, engine=cpu]
        kernel_name = a
        gpu_sim_cycle = 100
        gpu_tot_sim_insn = 1000
        gpu_ipc = 10.0
        kernel_name = b
        gpu_sim_cycle = 50
        gpu_tot_sim_insn = 1500
        gpu_ipc = 10.0
        kernel_name = a
        gpu_sim_cycle = 70
        gpu_tot_sim_insn = 2100
        GPGPU-Sim: *** exit detected ***
        """)
    spec = {"collect_aggregate": [r"gpu_tot_sim_insn\s*=\s*(.*)"], "collect_abs": [r"gpu_sim_cycle\s*=\s*(.*)"],
            "collect_rates": []}
    ks, order = get_stats.parse_output(out, spec, per_kernel=True, kernel_instance=True)
    assert order == ["a--0", "b--0", "a--1"]
    assert ks["a--0"][spec["collect_aggregate"][0]] == "1000"
    assert ks["b--0"][spec["collect_aggregate"][0]] == "500"
    assert ks["a--1"][spec["collect_aggregate"][0]] == "600"
    assert ks["a--1"][spec["collect_abs"][0]] == "70"
    ks, order = get_stats.parse_output(out, spec, per_kernel=True, kernel_instance=False)
    assert ks["a"]["k-count"] == "2" and ks["a"][spec["collect_aggregate"][0]] == "1600"
    ks, order = get_stats.parse_output(out, spec, per_kernel=False, kernel_instance=False)
    assert ks["final_kernel"][spec["collect_aggregate"][0]] == "2100"
    assert ks["final_kernel"]["Accel-Sim-build"].startswith("Accel-Sim-AMD")


def test_end_to_end_local_launch(native, tmp_path):
    """Launch a 2-app x 2-config grid on the local manager, wait, collect stats."""
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    traces = tmp_path / "traces"
    rodinia.write_app(str(traces / "vectoradd" / "NO_ARGS" / "traces"), [rodinia.vectoradd(8192)])
    rodinia.write_app(str(traces / "pathfinder" / "100_4_2" / "traces"), rodinia.pathfinder(100 * 16, 4, 2))
    ydir = tmp_path / "yml"
    (ydir / "apps").mkdir(parents=True)
    (ydir / "configs").mkdir()
    (ydir / "apps" / "define-tiny.yml").write_text(textwrap.dedent("""\
        tiny:
            exec_dir: ""
            data_dirs: ""
            execs:
                - vectoradd:
                    - args:
                - pathfinder:
                    - args: 100 4 2
        """))
    env = dict(os.environ, ASIM_YAML_PATH=str(ydir), ASIM_JOB_LOGDIR=str(tmp_path / "logs"),
               PROCMAN_STATE=str(tmp_path / "procman.json"), ASIM_CONFIG_ROOT=str(tmp_path / "cfgs"))
    jl = os.path.dirname(common.__file__)
    run = str(tmp_path / "run")
    r = subprocess.run([sys.executable, os.path.join(jl, "run_simulations.py"), "-B", "tiny", "-C",
                        "QV100-SASS,QV100-SASS-LRR", "-T", str(traces), "-N", "e2e", "-l", "local", "-r", run,
                        "-c", "2"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("submitted") == 4
    cfg = open(os.path.join(run, "pathfinder", "100_4_2", "QV100-SASS-LRR", "gpgpusim.config")).read()
    assert "-gpgpu_scheduler lrr" in cfg and "# Accel-Sim Parameters" in cfg
    stats_csv = str(tmp_path / "stats.csv")
    r = subprocess.run([sys.executable, os.path.join(jl, "monitor_func_test.py"), "-N", "e2e", "-r", run, "-S", "0.5",
                        "-T", "300", "-s", stats_csv], env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "All jobs passed" in r.stdout
    blocks = get_stats.parse_csv_blocks(open(stats_csv).read())
    cyc = blocks[r"gpu_tot_sim_cycle\s*=\s*(.*)"]
    assert set(cyc) == {"vectoradd/NO_ARGS--final_kernel", "pathfinder/100_4_2--final_kernel"}
    for row in cyc.values():
        assert int(row["QV100-SASS"]) > 0 and int(row["QV100-SASS-LRR"]) > 0
    # per-kernel, configs as rows
    r = subprocess.run([sys.executable, os.path.join(jl, "get_stats.py"), "-N", "e2e", "-r", run, "-K", "-R"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "CFG," in r.stdout and "pathfinder/100_4_2--" in r.stdout
    r = subprocess.run([sys.executable, os.path.join(jl, "job_status.py"), "-N", "e2e", "-r", run], env=env,
                       capture_output=True, text=True, timeout=120)
    assert "4/4 passed" in r.stdout, r.stdout
