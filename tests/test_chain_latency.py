"""Dependent-chain latency self-consistency of the tuner (tuner.py
_latency_self_consistency): ub_alu / ub_lds time one wave's dependent chain,
so after tuning the simulated twin of that chain must last exactly the
measured latency (the pipeline's own stages are taken out of the option)."""
import os
import shutil

import pytest

from accel_sim_framework_distributed_amd.tuner import tuner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "configs", "tuned", "AMD_Instinct_MI355X")


def _read(d):
    cfg = {}
    for fn in ("gpgpusim.config", "trace.config"):
        for line in open(os.path.join(d, fn)):
            t = line.split(None, 1)
            if len(t) == 2 and t[0].startswith("-"):
                cfg[t[0]] = t[1].strip()
    return cfg


@pytest.mark.timeout(300)
def test_chain_twin_matches_measured(tmp_path):
    pytest.importorskip("accel_sim_framework_distributed_amd._native")
    out = str(tmp_path / "cfg")
    shutil.copytree(CFG, out)
    cfg = _read(out)
    # the raw measurements of the MI355X run (TUNING.md): LDS 60, FMA 8, f64 FMA 7
    cfg["-gpgpu_smem_latency"] = "60"
    cfg["-trace_opcode_latency_initiation_sp"] = "8,2"
    cfg["-trace_opcode_latency_initiation_int"] = "8,2"
    cfg["-trace_opcode_latency_initiation_dp"] = "7,2"
    cfg["-gpgpu_l1_latency"] = "120"
    from accel_sim_framework_distributed_amd.models import presets
    presets.write_config(cfg, out, power_preset="MI355X")
    before = tuner.simulated_chain_latency(out, "ds_read_b32")
    assert before > 60  # the pipeline adds its own stages
    applied = {}
    notes = tuner._latency_self_consistency(out, cfg, applied, "MI355X")
    assert notes and "-gpgpu_smem_latency" in applied
    assert int(applied["-gpgpu_smem_latency"]) < 60
    assert applied["-trace_opcode_latency_initiation_int"] == applied["-trace_opcode_latency_initiation_sp"]
    assert tuner.simulated_chain_latency(out, "ds_read_b32") == pytest.approx(60, abs=1)
    assert tuner.simulated_chain_latency(out, "v_fma_f32") == pytest.approx(8, abs=1)
    assert tuner.simulated_chain_latency(out, "v_fma_f64") == pytest.approx(7, abs=1)
    assert tuner.simulated_chain_latency(out, "global_load_dword") == pytest.approx(120, abs=1)
