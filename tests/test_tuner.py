

def test_l1_port_granule_fit_from_strided_loads():
    """ub_l1_stride on MI355X: one 32 B sector per cycle (the tuner picks
    -sim_l1_port_granule 32 at the fitted 32 B/clk port)."""
    from accel_sim_framework_distributed_amd.tuner import tuner as T
    m = {4: 9.68, 8: 16.67, 16: 32.31, 32: 64.51, 64: 64.38, 128: 64.5}
    g, err, errs = T.fit_l1_port_granule(m, 32)
    assert g == 32 and err < 0.05 and errs[0] > 0.3
    assert T.l1_data_cycles(16, 32, 0) == 8 and T.l1_data_cycles(16, 32, 32) == 32


def test_sweep_address_mappings_match_reference_and_tuned_config():
    """The sweep's 32B / 256B address mappings are the reference's strings
    (define-standard-cfgs.yml:147-151); the tuned MI355X config uses the 256B
    one, so the sweep's 256B point is that config's own mapping."""
    import os
    from accel_sim_framework_distributed_amd.parallel.sweep import EXTRA_FLAGS
    m256 = EXTRA_FLAGS["256B"]["-gpgpu_mem_addr_mapping"]
    m32 = EXTRA_FLAGS["32B"]["-gpgpu_mem_addr_mapping"]
    assert m256 == "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCB.CCCSSSSS"
    assert m32 == "dramid@5;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCC.BCCSSSSS"
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "tuned",
                       "AMD_Instinct_MI355X", "gpgpusim.config")
    lines = [l.split(None, 1)[1].strip() for l in open(cfg) if l.startswith("-gpgpu_mem_addr_mapping")]
    assert lines == [m256]


def test_job_launching_registry_mappings_match_the_sweep():
    """define-standard-cfgs.yml's 32B / 256B extras carry the same (reference)
    mapping strings as the sweep, and GPU_ENGINE selects the MI355X engine."""
    import os
    import yaml
    from accel_sim_framework_distributed_amd.parallel.sweep import EXTRA_FLAGS
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "accel_sim_framework_distributed_amd",
                     "job_launching", "configs", "define-standard-cfgs.yml")
    y = yaml.safe_load(open(p))
    for k in ("32B", "256B"):
        assert y[k]["extra_params"] == "-gpgpu_mem_addr_mapping " + EXTRA_FLAGS[k]["-gpgpu_mem_addr_mapping"]
    assert y["GPU_ENGINE"]["extra_params"] == "-sim_engine gpu"


def test_sweep_gpu_end_declines_tail_jobs():
    """Node placement: a GPU slot stops taking jobs once the host cores would
    finish the next one sooner than the GPU (the step's tail)."""
    from accel_sim_framework_distributed_amd.parallel.sweep import SweepRunner
    r = SweepRunner.__new__(SweepRunner)
    r.ratio = {"fast": 0.5, "slow": 4.0}
    r.cpu_s = {"fast": 1.0, "slow": 1.0}
    job = lambda a: (a, None, "c", {})
    many = [job("slow")] * 40
    # plenty queued for 4 host cores (drain 10 s): a 4 s GPU job is worth taking
    assert r.gpu_takes(job("slow"), many, cslots=4)
    # two left for 4 cores (drain 0.5 s): the host core takes it in 1 s, the GPU in 4 s
    assert not r.gpu_takes(job("slow"), many[:2], cslots=4)
    # GPU-friendly jobs always go to the GPU; GPU-only sweeps never decline
    assert r.gpu_takes(job("fast"), [job("fast")], cslots=4)
    assert r.gpu_takes(job("slow"), [job("slow")], cslots=0)
