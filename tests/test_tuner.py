

def test_l1_port_granule_fit_from_strided_loads():
    """ub_l1_stride on MI355X: one 32 B sector per cycle (the tuner picks
    -sim_l1_port_granule 32 at the fitted 32 B/clk port)."""
    from accel_sim_framework_distributed_amd.tuner import tuner as T
    m = {4: 9.68, 8: 16.67, 16: 32.31, 32: 64.51, 64: 64.38, 128: 64.5}
    g, err, errs = T.fit_l1_port_granule(m, 32)
    assert g == 32 and err < 0.05 and errs[0] > 0.3
    assert T.l1_data_cycles(16, 32, 0) == 8 and T.l1_data_cycles(16, 32, 32) == 32
