"""Simulated-GPU presets (the "models" of this framework).

Each preset is a dict of gpgpusim.config / trace.config options describing a
GPU micro-architecture.  ``write_config`` renders it into the two-file layout
the reference uses (``gpgpusim.config`` + ``trace.config``, README.md:142-145),
so existing tools and run directories keep working.

Hardware values for the NVIDIA parts follow the public descriptions encoded in
the reference's tested configs (gpu-simulator/gpgpu-sim/configs/tested-cfgs/
SM7_QV100/gpgpusim.config and gpu-simulator/configs/tested-cfgs/*/trace.config);
``MI355X`` is this project's CDNA4 model (256 CUs in 8 XCDs, wave64, 4 SIMD32
per CU, 160 KB LDS, 32 KB L1, 4 MB L2 per XCD, HBM3E).
"""
from __future__ import annotations

import copy
import os
from typing import Dict, Iterable, Tuple

# options that belong in trace.config (trace-frontend latencies / units)
_TRACE_KEYS = (
    "-trace_opcode_latency_initiation_int",
    "-trace_opcode_latency_initiation_sp",
    "-trace_opcode_latency_initiation_dp",
    "-trace_opcode_latency_initiation_sfu",
    "-trace_opcode_latency_initiation_tensor",
)


def _volta_common() -> Dict[str, str]:
    return {
        # functional-sim flags still carried by tested configs
        "-gpgpu_ptx_instruction_classification": "0",
        "-gpgpu_ptx_sim_mode": "0",
        "-gpgpu_ptx_force_max_capability": "70",
        "-gpgpu_ptx_convert_to_ptxplus": "0",
        "-gpgpu_ptx_save_converted_ptxplus": "0",
        # device limits
        "-gpgpu_stack_size_limit": "1024",
        "-gpgpu_heap_size_limit": "8388608",
        "-gpgpu_runtime_sync_depth_limit": "2",
        "-gpgpu_runtime_pending_launch_count_limit": "2048",
        "-gpgpu_kernel_launch_latency": "5000",
        "-gpgpu_TB_launch_latency": "0",
        "-gpgpu_max_concurrent_kernel": "128",
        "-gpgpu_compute_capability_major": "7",
        "-gpgpu_compute_capability_minor": "0",
        # topology
        "-gpgpu_n_clusters": "80",
        "-gpgpu_n_cores_per_cluster": "1",
        "-gpgpu_n_mem": "32",
        "-gpgpu_n_sub_partition_per_mchannel": "2",
        "-gpgpu_clock_gated_lanes": "1",
        "-gpgpu_clock_domains": "1132.0:1132.0:1132.0:850.0",
        # core
        "-gpgpu_shader_registers": "65536",
        "-gpgpu_registers_per_block": "65536",
        "-gpgpu_occupancy_sm_number": "70",
        "-gpgpu_shader_core_pipeline": "2048:32",
        "-gpgpu_shader_cta": "32",
        "-gpgpu_simd_model": "1",
        "-gpgpu_pipeline_widths": "4,4,4,4,4,4,4,4,4,4,8,4,4",
        "-gpgpu_num_sp_units": "4",
        "-gpgpu_num_sfu_units": "4",
        "-gpgpu_num_dp_units": "4",
        "-gpgpu_num_int_units": "4",
        "-gpgpu_tensor_core_avail": "1",
        "-gpgpu_num_tensor_core_units": "4",
        "-ptx_opcode_latency_int": "4,13,4,5,145,21",
        "-ptx_opcode_initiation_int": "2,2,2,2,8,4",
        "-ptx_opcode_latency_fp": "4,13,4,5,39",
        "-ptx_opcode_initiation_fp": "2,2,2,2,4",
        "-ptx_opcode_latency_dp": "8,19,8,8,330",
        "-ptx_opcode_initiation_dp": "4,4,4,4,130",
        "-ptx_opcode_latency_sfu": "100",
        "-ptx_opcode_initiation_sfu": "8",
        "-ptx_opcode_latency_tesnor": "64",
        "-ptx_opcode_initiation_tensor": "64",
        "-gpgpu_sub_core_model": "1",
        "-gpgpu_enable_specialized_operand_collector": "0",
        "-gpgpu_operand_collector_num_units_gen": "8",
        "-gpgpu_operand_collector_num_in_ports_gen": "8",
        "-gpgpu_operand_collector_num_out_ports_gen": "8",
        "-gpgpu_num_reg_banks": "16",
        "-gpgpu_reg_file_port_throughput": "2",
        "-gpgpu_shmem_num_banks": "32",
        "-gpgpu_shmem_limited_broadcast": "0",
        "-gpgpu_shmem_warp_parts": "1",
        "-gpgpu_coalesce_arch": "70",
        "-gpgpu_num_sched_per_core": "4",
        "-gpgpu_scheduler": "lrr",
        "-gpgpu_max_insn_issue_per_warp": "1",
        "-gpgpu_dual_issue_diff_exec_units": "1",
        # L1 / shared
        "-gpgpu_adaptive_cache_config": "1",
        "-gpgpu_shmem_option": "0,8,16,32,64,96",
        "-gpgpu_unified_l1d_size": "128",
        "-gpgpu_l1_banks": "4",
        "-gpgpu_cache:dl1": "S:4:128:64,L:T:m:L:L,A:512:8,16:0,32",
        "-gpgpu_l1_cache_write_ratio": "25",
        "-gpgpu_l1_latency": "20",
        "-gpgpu_gmem_skip_L1D": "0",
        "-gpgpu_flush_l1_cache": "1",
        "-gpgpu_n_cluster_ejection_buffer_size": "32",
        "-gpgpu_shmem_size": "98304",
        "-gpgpu_shmem_sizeDefault": "98304",
        "-gpgpu_shmem_per_block": "65536",
        "-gpgpu_smem_latency": "20",
        # L2 / memory
        "-gpgpu_cache:dl2": "S:32:128:24,L:B:m:L:P,A:192:4,32:0,32",
        "-gpgpu_cache:dl2_texture_only": "0",
        "-gpgpu_dram_partition_queues": "64:64:64:64",
        "-gpgpu_perf_sim_memcpy": "1",
        "-gpgpu_memory_partition_indexing": "2",
        "-gpgpu_cache:il1": "N:64:128:16,L:R:f:N:L,S:2:48,4",
        "-gpgpu_inst_fetch_throughput": "4",
        "-gpgpu_tex_cache:l1": "N:4:128:256,L:R:m:N:L,T:512:8,128:2",
        "-gpgpu_const_cache:l1": "N:128:64:8,L:R:f:N:L,S:2:64,4",
        "-gpgpu_perfect_inst_const_cache": "1",
        # interconnect (local crossbar)
        "-network_mode": "2",
        "-icnt_in_buffer_limit": "512",
        "-icnt_out_buffer_limit": "512",
        "-icnt_subnets": "2",
        "-icnt_flit_size": "40",
        "-icnt_arbiter_algo": "1",
        "-gpgpu_l2_rop_latency": "160",
        "-dram_latency": "100",
        # DRAM (HBM2)
        "-gpgpu_dram_scheduler": "1",
        "-gpgpu_frfcfs_dram_sched_queue_size": "64",
        "-gpgpu_dram_return_queue_size": "192",
        "-gpgpu_n_mem_per_ctrlr": "1",
        "-gpgpu_dram_buswidth": "16",
        "-gpgpu_dram_burst_length": "2",
        "-dram_data_command_freq_ratio": "2",
        "-gpgpu_mem_address_mask": "1",
        "-gpgpu_mem_addr_mapping": "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCB.CCCSSSSS",
        "-gpgpu_dram_timing_opt": '"nbk=16:CCD=1:RRD=3:RCD=12:RAS=28:RP=12:RC=40:CL=12:WL=2:CDLR=3:WR=10:nbkgrp=4:CCDL=2:RTPL=3"',
        "-dram_dual_bus_interface": "1",
        "-dram_bnk_indexing_policy": "0",
        "-dram_bnkgrp_indexing_policy": "1",
        # stats
        "-gpgpu_memlatency_stat": "14",
        "-gpgpu_runtime_stat": "500",
        "-enable_ptx_file_line_stats": "1",
        "-visualizer_enabled": "0",
        # trace frontend
        "-trace_opcode_latency_initiation_int": "4,2",
        "-trace_opcode_latency_initiation_sp": "4,2",
        "-trace_opcode_latency_initiation_dp": "8,4",
        "-trace_opcode_latency_initiation_sfu": "20,8",
        "-trace_opcode_latency_initiation_tensor": "8,4",
        "-specialized_unit_1": "1,4,4,4,4,BRA",
        "-trace_opcode_latency_initiation_spec_op_1": "4,4",
        "-specialized_unit_2": "1,4,200,4,4,TEX",
        "-trace_opcode_latency_initiation_spec_op_2": "200,4",
        "-specialized_unit_3": "1,4,8,4,4,TENSOR",
        "-trace_opcode_latency_initiation_spec_op_3": "2,2",
    }


def _qv100() -> Dict[str, str]:
    return _volta_common()


def _gv100() -> Dict[str, str]:
    c = _volta_common()
    c["-gpgpu_clock_domains"] = "1447.0:1447.0:1447.0:850.0"
    return c


def _titanv() -> Dict[str, str]:
    c = _volta_common()
    c["-gpgpu_n_mem"] = "24"
    c["-gpgpu_clock_domains"] = "1200.0:1200.0:1200.0:850.0"
    return c


def _rtx2060() -> Dict[str, str]:
    c = _volta_common()
    c.update({
        "-gpgpu_compute_capability_minor": "5",
        "-gpgpu_ptx_force_max_capability": "75",
        "-gpgpu_n_clusters": "30",
        "-gpgpu_n_mem": "12",
        "-gpgpu_shader_core_pipeline": "1024:32",
        "-gpgpu_clock_domains": "1365.0:1365.0:1365.0:3500.0",
        "-gpgpu_unified_l1d_size": "96",
        "-gpgpu_shmem_option": "32,64",
        "-gpgpu_shmem_size": "65536",
        "-gpgpu_shmem_sizeDefault": "65536",
        "-gpgpu_shader_cta": "16",
        "-gpgpu_cache:dl2": "S:64:128:16,L:B:m:L:P,A:192:4,32:0,32",
        "-gpgpu_memory_partition_indexing": "0",
        "-gpgpu_dram_buswidth": "2",
        "-gpgpu_dram_burst_length": "16",
        "-dram_data_command_freq_ratio": "4",
        "-dram_dual_bus_interface": "0",
        "-gpgpu_mem_addr_mapping": "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCC.BCCSSSSS",
        "-gpgpu_dram_timing_opt": '"nbk=16:CCD=4:RRD=10:RCD=20:RAS=50:RP=20:RC=62:CL=20:WL=8:CDLR=9:WR=20:nbkgrp=4:CCDL=4:RTPL=4"',
    })
    return c


def _rtx3070() -> Dict[str, str]:
    c = _rtx2060()
    c.update({
        "-gpgpu_compute_capability_major": "8",
        "-gpgpu_compute_capability_minor": "6",
        "-gpgpu_ptx_force_max_capability": "86",
        "-gpgpu_n_clusters": "46",
        "-gpgpu_n_mem": "16",
        "-gpgpu_shader_core_pipeline": "1536:32",
        "-gpgpu_clock_domains": "1132.0:1132.0:1132.0:3500.0",
        "-gpgpu_unified_l1d_size": "128",
        "-gpgpu_shmem_option": "0,8,16,32,64,100",
        "-gpgpu_shmem_size": "102400",
        "-gpgpu_shmem_sizeDefault": "102400",
    })
    return c


def _mi355x() -> Dict[str, str]:
    """CDNA4 / MI355X model: 256 CUs (8 XCDs x 32), wave64, 4 SIMD32 per CU.

    Per CU: 32 waves max, 512 VGPR x 64 lanes x 4 SIMDs of registers, 160 KB
    LDS (64 banks x 4 B), 32 KB vector L1 (128 B lines, 64 B sectors on
    hardware; modelled as 4 x 32 B sectors), MFMA per SIMD.  Memory: 8 HBM3E
    stacks x 16 channels = 128 channels with one L2 slice each (4 MB L2 per XCD =
    256 KB per slice), 2.4 GHz core clock, HBM3E at 8 TB/s aggregate.
    """
    c = _volta_common()
    c.update({
        "-gpgpu_compute_capability_major": "9",
        "-gpgpu_compute_capability_minor": "50",
        "-gpgpu_ptx_force_max_capability": "0",
        "-gpgpu_n_clusters": "256",
        "-gpgpu_n_cores_per_cluster": "1",
        # 8 HBM3E stacks x 16 channels; one L2 slice per channel (16 per XCD)
        "-gpgpu_n_mem": "128",
        "-gpgpu_n_sub_partition_per_mchannel": "1",
        "-gpgpu_clock_domains": "2400.0:2400.0:2400.0:1600.0",
        "-gpgpu_shader_core_pipeline": "2048:64",
        "-gpgpu_shader_registers": "131072",
        "-gpgpu_registers_per_block": "131072",
        "-gpgpu_shader_cta": "32",
        "-gpgpu_num_sched_per_core": "4",
        "-gpgpu_scheduler": "gto",
        "-gpgpu_shmem_num_banks": "64",
        "-gpgpu_shmem_size": "163840",
        "-gpgpu_shmem_sizeDefault": "163840",
        "-gpgpu_shmem_per_block": "163840",
        "-gpgpu_adaptive_cache_config": "0",
        "-gpgpu_unified_l1d_size": "0",
        "-gpgpu_cache:dl1": "S:64:128:4,L:T:m:L:L,A:256:8,16:0,32",
        # instruction cache: 64 KB shared by a CU pair -> 32 KB per CU, modelled
        # (not perfect) because small kernels pay their cold misses
        "-gpgpu_perfect_inst_const_cache": "0",
        # hipMemcpy H2D goes through SDMA to HBM, not through the XCD L2s
        "-gpgpu_perf_sim_memcpy": "0",
        "-gpgpu_cache:il1": "N:64:128:4,L:R:f:N:L,S:4:64,4",
        "-gpgpu_l1_latency": "120",
        "-gpgpu_smem_latency": "64",
        "-gpgpu_cache:dl2": "S:128:128:8,L:B:m:L:P,A:192:4,32:0,32",
        "-gpgpu_l2_rop_latency": "200",
        "-dram_latency": "300",
        "-gpgpu_memory_partition_indexing": "2",
        "-gpgpu_dram_buswidth": "32",
        "-gpgpu_dram_burst_length": "2",
        "-dram_data_command_freq_ratio": "2",
        "-gpgpu_mem_addr_mapping": "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCB.CCCSSSSS",
        "-icnt_flit_size": "64",
        "-trace_opcode_latency_initiation_int": "4,2",
        "-trace_opcode_latency_initiation_sp": "4,2",
        "-trace_opcode_latency_initiation_dp": "8,4",
        "-trace_opcode_latency_initiation_sfu": "16,8",
        "-trace_opcode_latency_initiation_tensor": "32,16",
    })
    return c


PRESETS = {
    "QV100": _qv100,
    "GV100": _gv100,
    "TITANV": _titanv,
    "RTX2060": _rtx2060,
    "RTX3070": _rtx3070,
    "MI355X": _mi355x,
}


def get_preset(name: str) -> Dict[str, str]:
    key = name.upper().replace("-SASS", "").replace("SM7_", "").replace("SM75_", "").replace("SM86_", "")
    if key not in PRESETS:
        raise KeyError(f"unknown GPU preset {name!r}; known: {sorted(PRESETS)}")
    return copy.deepcopy(PRESETS[key]())


def render(opts: Dict[str, str], keys: Iterable[str]) -> str:
    lines = []
    for k in keys:
        v = opts[k]
        lines.append(f"{k} {v}")
    return "\n".join(lines) + "\n"


def split_config(opts: Dict[str, str]) -> Tuple[Dict[str, str], Dict[str, str]]:
    trace = {k: v for k, v in opts.items()
             if k in _TRACE_KEYS or k.startswith("-trace_opcode_latency_initiation_spec_op_")
             or k.startswith("-specialized_unit_")}
    gpgpu = {k: v for k, v in opts.items() if k not in trace}
    return gpgpu, trace


def write_config(name_or_opts, out_dir: str, extra: Dict[str, str] | None = None,
                 power_preset: str | None = None) -> Tuple[str, str]:
    """Write gpgpusim.config + trace.config for a preset; returns both paths.
    ``power_preset`` names the preset whose default AccelWattch XMLs go next
    to a custom option dict (default: the preset's own)."""
    opts = get_preset(name_or_opts) if isinstance(name_or_opts, str) else dict(name_or_opts)
    if extra:
        opts.update(extra)
    gp, tr = split_config(opts)
    os.makedirs(out_dir, exist_ok=True)
    p1 = os.path.join(out_dir, "gpgpusim.config")
    p2 = os.path.join(out_dir, "trace.config")
    with open(p1, "w") as f:
        f.write("# generated by accel_sim_framework_distributed_amd.models.presets\n")
        f.write(render(gp, sorted(gp)))
    with open(p2, "w") as f:
        f.write(render(tr, sorted(tr)))
    # AccelWattch XMLs next to the configs (SIM / HW / HYBRID modes share the
    # uncalibrated defaults until power.calibrate rewrites them)
    from ..power.xmlcfg import default_params, write_xml
    pname = power_preset or (name_or_opts if isinstance(name_or_opts, str) else "custom")
    for mode in ("sim", "hw", "hybrid"):
        xp = os.path.join(out_dir, f"accelwattch_sass_{mode}.xml")
        if not os.path.exists(xp):
            write_xml(xp, default_params(pname), comment=f"{pname} defaults (uncalibrated)")
    return p1, p2


def args_for(name_or_opts, extra: Dict[str, str] | None = None) -> list:
    """Flat argv list (no files) for a preset, for in-process simulators."""
    opts = get_preset(name_or_opts) if isinstance(name_or_opts, str) else dict(name_or_opts)
    if extra:
        opts.update(extra)
    argv = []
    for k, v in opts.items():
        if len(v) >= 2 and v[0] == '"' and v[-1] == '"':
            v = v[1:-1]
        argv += [k, v]
    return argv
