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
        # SM7_QV100/trace.config:1-5
        "-trace_opcode_latency_initiation_int": "2,2",
        "-trace_opcode_latency_initiation_sp": "2,2",
        "-trace_opcode_latency_initiation_dp": "8,4",
        "-trace_opcode_latency_initiation_sfu": "20,8",
        "-trace_opcode_latency_initiation_tensor": "2,2",
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
    # SM7_TITANV/gpgpusim.config + trace.config
    c.update({
        "-gpgpu_n_clusters": "40", "-gpgpu_n_cores_per_cluster": "2",
        "-ptx_opcode_latency_int": "4,13,4,5,145,32", "-gpgpu_num_reg_banks": "8", "-gpgpu_coalesce_arch": "60",
        "-dram_bnk_indexing_policy": "1", "-dram_seperate_write_queue_enable": "1",
        "-dram_write_queue_size": "128:108:32",
        "-trace_opcode_latency_initiation_tensor": "8,4", "-trace_opcode_latency_initiation_spec_op_3": "8,4",
        "-gpgpu_kernel_launch_latency": "0",  # not set in SM7_TITANV/gpgpusim.config: the option default
    })
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
    # SM75_RTX2060/gpgpusim.config + trace.config
    c.update({
        "-gpgpu_clock_domains": "1365:1365:1365:3500.5", "-gpgpu_occupancy_sm_number": "75",
        "-ptx_opcode_latency_int": "4,4,4,4,21", "-ptx_opcode_initiation_int": "2,2,2,2,2",
        "-ptx_opcode_latency_fp": "4,4,4,4,39", "-ptx_opcode_latency_dp": "64,64,64,64,330",
        "-ptx_opcode_initiation_dp": "64,64,64,64,130", "-ptx_opcode_latency_sfu": "21",
        "-gpgpu_num_reg_banks": "8", "-gpgpu_cache:dl1": "S:4:128:64,L:T:m:L:L,A:256:32,16:0,32",
        "-gpgpu_l1_latency": "32", "-gpgpu_shmem_per_block": "49152", "-gpgpu_smem_latency": "30",
        "-gpgpu_coalesce_arch": "75", "-gpgpu_l2_rop_latency": "194", "-dram_latency": "96",
        "-gpgpu_dram_timing_opt": '"nbk=16:CCD=4:RRD=12:RCD=24:RAS=55:RP=24:RC=78:CL=24:WL=8:CDLR=10:WR=24:nbkgrp=4:CCDL=6:RTPL=4"',
        "-trace_opcode_latency_initiation_dp": "64,64", "-trace_opcode_latency_initiation_sfu": "21,8",
        "-trace_opcode_latency_initiation_tensor": "16,16", "-specialized_unit_3": "1,4,16,4,4,TENSOR",
        "-trace_opcode_latency_initiation_spec_op_3": "16,16", "-specialized_unit_4": "1,4,4,4,4,UDP",
        "-trace_opcode_latency_initiation_spec_op_4": "4,1",
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
    # SM86_RTX3070/gpgpusim.config + trace.config
    c.update({
        "-gpgpu_clock_domains": "1132:1132:1132:3500.5", "-gpgpu_occupancy_sm_number": "86",
        "-gpgpu_shader_cta": "32", "-ptx_opcode_initiation_fp": "1,1,1,1,2",
        "-gpgpu_cache:dl1": "S:4:128:256,L:T:m:L:L,A:384:48,16:0,32", "-gpgpu_l1_latency": "39",
        "-gpgpu_smem_latency": "29", "-gpgpu_coalesce_arch": "86", "-gpgpu_memory_partition_indexing": "2",
        "-gpgpu_l2_rop_latency": "187", "-dram_latency": "254",
        "-trace_opcode_latency_initiation_sp": "2,1", "-trace_opcode_latency_initiation_tensor": "32,32",
        "-specialized_unit_3": "1,4,32,4,4,TENSOR", "-trace_opcode_latency_initiation_spec_op_3": "32,32",
    })
    return c


# ---- interconnect files for -network_mode 1 (Booksim/intersim2 format) ----
# Every tested pre-Volta config uses a single-stage butterfly (a crossbar with
# iSLIP allocation) sized to clusters + memory sub-partitions (reference
# configs/tested-cfgs/*/config_*_islip.icnt); the generator below writes the
# same parameter set for any node count / topology.
def icnt_params(k: int, topology: str = "fly", n: int = 1, flit_size: int = 40, **over) -> Dict[str, str]:
    p = {
        "use_map": "0", "flit_size": str(flit_size), "network_count": "2",
        "topology": topology, "k": str(k), "n": str(n), "routing_function": "dest_tag",
        "num_vcs": "1", "vc_buf_size": "64", "input_buffer_size": "256", "ejection_buffer_size": "64",
        "boundary_buffer_size": "64", "wait_for_tail_credit": "0", "vc_allocator": "islip",
        "sw_allocator": "islip", "alloc_iters": "1", "credit_delay": "0", "routing_delay": "0",
        "vc_alloc_delay": "1", "sw_alloc_delay": "1", "input_speedup": "1", "output_speedup": "1",
        "internal_speedup": "2.0", "traffic": "uniform", "sim_type": "gpgpusim", "injection_rate": "0.1",
        "subnets": "2", "read_request_subnet": "0", "read_reply_subnet": "1", "write_request_subnet": "0",
        "write_reply_subnet": "1",
    }
    p.update({kk: str(v) for kk, v in over.items()})
    return p


def render_icnt(params: Dict[str, str], title: str = "") -> str:
    lines = [f"// {title}" if title else "// generated by accel_sim_framework_distributed_amd.models.presets"]
    lines += [f"{k} = {v};" for k, v in params.items()]
    return "\n".join(lines) + "\n"


# preset -> (file name, booksim parameters)
ICNT_FILES: Dict[str, Tuple[str, Dict[str, str]]] = {
    "GTX480": ("config_fermi_islip.icnt", icnt_params(27)),
    "KEPLER_TITAN": ("config_kepler_islip.icnt", icnt_params(38)),
    "TITANX": ("config_pascal_islip.icnt", icnt_params(52)),
}


def _pre_volta_common() -> Dict[str, str]:
    """Fermi/Kepler/Pascal-era settings shared by the tested pre-Volta configs
    (SM2_GTX480, SM3_KEPLER_TITAN, SM6_TITANX gpgpusim.config)."""
    c = _volta_common()
    for k in [k for k in c if k.startswith("-specialized_unit_") or "_spec_op_" in k]:
        del c[k]
    # the pre-Volta tested configs leave the crossbar buffers at their defaults
    for k in ("-icnt_in_buffer_limit", "-icnt_out_buffer_limit"):
        c.pop(k, None)
    c.update({
        "-gpgpu_ignore_resources_limitation": "1",
        "-gpgpu_kernel_launch_latency": "0",
        "-gpgpu_tensor_core_avail": "0",
        "-gpgpu_num_tensor_core_units": "0",
        "-gpgpu_num_int_units": "0",
        "-gpgpu_num_dp_units": "0",
        "-gpgpu_sub_core_model": "0",
        "-gpgpu_adaptive_cache_config": "0",
        "-gpgpu_unified_l1d_size": "0",
        "-gpgpu_shmem_option": "0",
        "-gpgpu_l1_banks": "1",
        "-gpgpu_l1_cache_write_ratio": "0",
        "-gpgpu_gmem_skip_L1D": "1",
        "-gpgpu_scheduler": "gto",
        "-gpgpu_max_insn_issue_per_warp": "2",
        "-gpgpu_dual_issue_diff_exec_units": "1",
        "-gpgpu_memory_partition_indexing": "0",
        "-gpgpu_perfect_inst_const_cache": "0",
        "-gpgpu_cache:il1": "N:8:128:4,L:R:f:N:L,S:2:48,4",
        "-gpgpu_inst_fetch_throughput": "8",
        "-gpgpu_tex_cache:l1": "N:16:128:24,L:R:m:N:L,T:128:4,128:2",
        "-gpgpu_const_cache:l1": "N:128:64:2,L:R:f:N:L,S:2:64,4",
        "-gpgpu_dram_partition_queues": "32:32:32:32",
        "-gpgpu_l2_rop_latency": "120",
        "-dram_latency": "100",
        "-gpgpu_frfcfs_dram_sched_queue_size": "64",
        "-gpgpu_dram_return_queue_size": "64",
        "-gpgpu_dram_buswidth": "4",
        "-gpgpu_dram_burst_length": "8",
        "-dram_data_command_freq_ratio": "4",
        "-dram_dual_bus_interface": "0",
        "-gpgpu_mem_addr_mapping": "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCC.BCCSSSSS",
        "-gpgpu_dram_timing_opt": '"nbk=16:CCD=2:RRD=8:RCD=16:RAS=37:RP=16:RC=52:CL=16:WL=6:CDLR=7:WR=16:nbkgrp=4:CCDL=4:RTPL=3"',
        "-network_mode": "1",
        "-icnt_flit_size": "40",
        "-gpgpu_n_cluster_ejection_buffer_size": "32",
        "-gpgpu_flush_l1_cache": "1",
        "-gpgpu_l1_latency": "82",
        "-gpgpu_smem_latency": "24",
        "-trace_opcode_latency_initiation_int": "4,1",
        "-trace_opcode_latency_initiation_sp": "4,1",
        "-trace_opcode_latency_initiation_dp": "20,8",
        "-trace_opcode_latency_initiation_sfu": "20,4",
        "-trace_opcode_latency_initiation_tensor": "4,1",
    })
    return c


def _titanx() -> Dict[str, str]:
    """Pascal TITAN X (SM6_TITANX): 28 SMs, 12 GDDR5X channels x 2, fly(52) icnt."""
    c = _pre_volta_common()
    c.update({
        "-gpgpu_compute_capability_major": "6", "-gpgpu_compute_capability_minor": "1",
        "-gpgpu_ptx_force_max_capability": "61", "-gpgpu_occupancy_sm_number": "62",
        "-gpgpu_n_clusters": "28", "-gpgpu_n_mem": "12", "-gpgpu_n_sub_partition_per_mchannel": "2",
        "-gpgpu_clock_domains": "1417.0:1417.0:1417.0:2500.0",
        "-gpgpu_pipeline_widths": "4,0,0,4,4,4,0,0,4,4,8",
        "-gpgpu_num_sp_units": "4", "-gpgpu_num_sfu_units": "4",
        "-gpgpu_coalesce_arch": "61", "-gpgpu_l1_banks": "2",
        "-gpgpu_cache:dl1": "S:4:128:96,L:L:s:N:L,A:256:8,16:0,32",
        "-gpgpu_shmem_size": "98304", "-gpgpu_shmem_sizeDefault": "98304", "-gpgpu_shmem_per_block": "49152",
        "-gpgpu_cache:dl2": "S:64:128:16,L:B:m:L:P,A:256:64,16:0,32",
        "-gpgpu_memory_partition_indexing": "4",
        "-gpgpu_perfect_inst_const_cache": "1",
        "-gpgpu_kernel_launch_latency": "5000",
        "-gpgpu_mem_addr_mapping": "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCC.BCCSSSSS",
        "-inter_config_file": "config_pascal_islip.icnt",
    })
    # SM6_TITANX/gpgpusim.config
    c.update({
        "-ptx_opcode_latency_int": "4,13,4,5,145,32", "-ptx_opcode_initiation_int": "1,1,1,1,4,4",
        "-ptx_opcode_latency_fp": "4,13,4,4,39", "-ptx_opcode_initiation_fp": "1,2,1,1,4",
        "-ptx_opcode_initiation_dp": "8,8,8,8,130", "-ptx_opcode_initiation_sfu": "4", "-ptx_opcode_latency_sfu": "20",
        "-gpgpu_sub_core_model": "1",
        "-gpgpu_cache:dl1PrefL1": "S:4:128:96,L:L:s:N:L,A:256:8,16:0,32",
        "-gpgpu_cache:dl1PrefShared": "S:4:128:96,L:L:s:N:L,A:256:8,16:0,32",
        "-gpgpu_shmem_size_PrefL1": "98304", "-gpgpu_shmem_size_PrefShared": "98304",
    })
    return c


def _kepler_titan() -> Dict[str, str]:
    """Kepler GTX TITAN (SM3_KEPLER_TITAN): 14 SMX, 12 channels x 2, fly(38) icnt."""
    c = _pre_volta_common()
    c.update({
        "-gpgpu_compute_capability_major": "3", "-gpgpu_compute_capability_minor": "5",
        "-gpgpu_ptx_force_max_capability": "35", "-gpgpu_occupancy_sm_number": "62",
        "-gpgpu_n_clusters": "14", "-gpgpu_n_mem": "12", "-gpgpu_n_sub_partition_per_mchannel": "2",
        "-gpgpu_clock_domains": "837.0:837.0:837.0:1502.0",
        "-gpgpu_shader_cta": "16",
        "-gpgpu_pipeline_widths": "6,4,0,2,1,6,4,0,2,1,12",
        "-gpgpu_num_sp_units": "6", "-gpgpu_num_sfu_units": "2", "-gpgpu_num_dp_units": "4",
        "-gpgpu_enable_specialized_operand_collector": "1",
        "-gpgpu_operand_collector_num_units_sp": "12", "-gpgpu_operand_collector_num_units_sfu": "6",
        "-gpgpu_operand_collector_num_units_mem": "8", "-gpgpu_operand_collector_num_units_dp": "6",
        "-gpgpu_operand_collector_num_units_gen": "0",
        "-gpgpu_coalesce_arch": "35", "-gpgpu_dual_issue_diff_exec_units": "0",
        "-gpgpu_cache:dl1": "S:4:128:32,L:L:s:N:L,A:256:8,16:0,32",
        "-gpgpu_shmem_size": "49152", "-gpgpu_shmem_sizeDefault": "49152", "-gpgpu_shmem_per_block": "49152",
        "-gpgpu_cache:dl2": "S:32:128:16,L:B:m:L:P,A:256:64,16:0,32",
        "-gpgpu_clock_gated_lanes": "0",
        "-inter_config_file": "config_kepler_islip.icnt",
        "-trace_opcode_latency_initiation_dp": "20,2",
        "-trace_opcode_latency_initiation_sfu": "200,2",
    })
    # SM3_KEPLER_TITAN/gpgpusim.config
    c.update({
        "-ptx_opcode_latency_int": "4,13,4,5,145,32", "-ptx_opcode_initiation_int": "1,1,1,1,4,4",
        "-ptx_opcode_initiation_fp": "1,2,1,1,4", "-ptx_opcode_initiation_dp": "2,8,8,8,130",
        "-ptx_opcode_initiation_sfu": "2", "-ptx_opcode_latency_sfu": "200",
        "-gpgpu_operand_collector_num_in_ports_sp": "2", "-gpgpu_operand_collector_num_out_ports_sp": "2",
        "-gpgpu_operand_collector_num_in_ports_sfu": "2", "-gpgpu_operand_collector_num_out_ports_sfu": "2",
        "-gpgpu_operand_collector_num_in_ports_mem": "1", "-gpgpu_operand_collector_num_out_ports_mem": "1",
        "-gpgpu_operand_collector_num_in_ports_dp": "1", "-gpgpu_operand_collector_num_out_ports_dp": "1",
        "-gpgpu_cache:dl1PrefL1": "S:4:128:96,L:L:s:N:L,A:256:8,16:0,32",
        "-gpgpu_cache:dl1PrefShared": "S:4:128:32,L:L:s:N:L,A:256:8,16:0,32",
        "-gpgpu_shmem_size_PrefL1": "16384", "-gpgpu_shmem_size_PrefShared": "49152", "-smem_latency": "24",
    })
    return c


def _gtx480() -> Dict[str, str]:
    """Fermi GTX 480 (SM2_GTX480): 15 SMs, 6 GDDR5 channels x 2, fly(27) icnt."""
    c = _pre_volta_common()
    c.update({
        "-gpgpu_compute_capability_major": "2", "-gpgpu_compute_capability_minor": "0",
        "-gpgpu_ptx_force_max_capability": "20", "-gpgpu_occupancy_sm_number": "20",
        "-gpgpu_n_clusters": "15", "-gpgpu_n_mem": "6", "-gpgpu_n_sub_partition_per_mchannel": "2",
        "-gpgpu_clock_domains": "700.0:700.0:700.0:924.0",
        "-gpgpu_shader_registers": "32768", "-gpgpu_registers_per_block": "32768",
        "-gpgpu_shader_core_pipeline": "1536:32", "-gpgpu_shader_cta": "8",
        "-gpgpu_pipeline_widths": "2,0,0,1,1,2,0,0,1,1,2",
        "-gpgpu_num_sp_units": "2", "-gpgpu_num_sfu_units": "1",
        "-gpgpu_num_sched_per_core": "2", "-gpgpu_max_insn_issue_per_warp": "1",
        "-gpgpu_enable_specialized_operand_collector": "1",
        "-gpgpu_operand_collector_num_units_sp": "6", "-gpgpu_operand_collector_num_units_sfu": "8",
        "-gpgpu_operand_collector_num_units_mem": "2", "-gpgpu_operand_collector_num_units_gen": "0",
        "-gpgpu_coalesce_arch": "20", "-gpgpu_ignore_resources_limitation": "0",
        "-gpgpu_cache:dl1": "N:32:128:4,L:L:m:N:H,S:64:8,8",
        "-gpgpu_gmem_skip_L1D": "0", "-gpgpu_l1_latency": "35", "-gpgpu_smem_latency": "26",
        "-gpgpu_shmem_size": "49152", "-gpgpu_shmem_sizeDefault": "49152", "-gpgpu_shmem_per_block": "49152",
        "-gpgpu_cache:dl2": "S:64:128:8,L:B:m:L:L,A:256:4,4:0,32",
        "-gpgpu_cache:il1": "N:4:128:4,L:R:f:N:L,S:2:32,4",
        "-gpgpu_const_cache:l1": "N:64:64:2,L:R:f:N:L,S:2:32,4",
        "-gpgpu_dram_partition_queues": "64:64:64:64",
        "-gpgpu_dram_return_queue_size": "116",
        "-gpgpu_n_mem_per_ctrlr": "2",
        "-gpgpu_mem_addr_mapping": "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.BBBCCCCB.CCSSSSSS",
        "-gpgpu_dram_timing_opt": '"nbk=16:CCD=2:RRD=6:RCD=12:RAS=28:RP=12:RC=40:CL=12:WL=4:CDLR=5:WR=12:nbkgrp=4:CCDL=3:RTPL=2"',
        "-gpgpu_clock_gated_lanes": "0",
        "-inter_config_file": "config_fermi_islip.icnt",
    })
    # SM2_GTX480/gpgpusim.config
    c.update({
        "-ptx_opcode_latency_int": "4,13,4,5,145,32", "-ptx_opcode_initiation_int": "1,2,2,1,8,4",
        "-ptx_opcode_initiation_fp": "1,2,1,1,4", "-ptx_opcode_initiation_dp": "8,16,8,8,130",
        "-gpgpu_tex_cache:l1": "N:4:128:24,L:R:m:N:L,T:128:4,128:2",
        "-gpgpu_operand_collector_num_in_ports_sp": "2", "-gpgpu_operand_collector_num_out_ports_sp": "2",
        # no trace.config for SM2_GTX480 and no fetch throughput line: option defaults
        "-gpgpu_inst_fetch_throughput": "1",
        "-trace_opcode_latency_initiation_int": "4,1", "-trace_opcode_latency_initiation_sp": "4,1",
        "-trace_opcode_latency_initiation_dp": "4,1", "-trace_opcode_latency_initiation_sfu": "4,1",
        "-trace_opcode_latency_initiation_tensor": "4,1",
    })
    return c


def _rtx2060_s() -> Dict[str, str]:
    """RTX 2060 SUPER (SM75_RTX2060_S): 34 SMs at 1905 MHz, 16 GDDR6 channels."""
    c = _rtx2060()
    c.update({
        "-gpgpu_n_clusters": "34", "-gpgpu_n_mem": "16",
        "-gpgpu_clock_domains": "1905.0:1905.0:1905.0:3500.0",
        "-gpgpu_shader_cta": "32", "-gpgpu_num_reg_banks": "16",
        "-gpgpu_pipeline_widths": "4,0,4,4,4,4,0,4,4,4,8,4,4",
        "-gpgpu_adaptive_cache_config": "0",
        "-gpgpu_cache:dl1": "S:1:128:512,L:L:s:N:L,A:256:8,16:0,32",
        "-gpgpu_shmem_per_block": "65536",
        "-gpgpu_l1_latency": "20", "-gpgpu_smem_latency": "20", "-gpgpu_l2_rop_latency": "160",
        "-dram_latency": "100",
        "-trace_opcode_latency_initiation_int": "2,2", "-trace_opcode_latency_initiation_sp": "2,2",
        "-trace_opcode_latency_initiation_dp": "64,64", "-trace_opcode_latency_initiation_sfu": "21,8",
        "-trace_opcode_latency_initiation_tensor": "16,16",
        "-specialized_unit_3": "1,4,16,4,4,TENSOR",
        "-trace_opcode_latency_initiation_spec_op_3": "16,16",
        "-specialized_unit_4": "1,4,4,4,4,UDP",
        "-trace_opcode_latency_initiation_spec_op_4": "4,1",
    })
    # SM75_RTX2060_S/gpgpusim.config: the Volta-style FU latencies
    c.update({
        "-gpgpu_occupancy_sm_number": "75", "-gpgpu_coalesce_arch": "75", "-gpgpu_num_dp_units": "0",
        "-ptx_opcode_latency_int": "4,13,4,5,145,32", "-ptx_opcode_initiation_int": "2,2,2,2,8,4",
        "-ptx_opcode_latency_fp": "4,13,4,5,39", "-ptx_opcode_latency_dp": "8,19,8,8,330",
        "-ptx_opcode_initiation_dp": "4,4,4,4,130", "-ptx_opcode_latency_sfu": "100",
        "-gpgpu_dram_timing_opt": '"nbk=16:CCD=4:RRD=10:RCD=20:RAS=50:RP=20:RC=62:CL=20:WL=8:CDLR=9:WR=20:nbkgrp=4:CCDL=4:RTPL=4"',
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
        # one wave issues an instruction every ~5.5 cycles (ub_wave_issue)
        "-gpgpu_warp_issue_interval": "5",
        "-gpgpu_scheduler": "gto",
        "-gpgpu_shmem_num_banks": "64",
        # a wave's instruction buffer reads the SQC once per 32 B block it enters
        # (SQC_ICACHE_HITS + MISSES vs the traced PCs of the Rodinia suite)
        "-gpgpu_inst_fetch_block_bytes": "32",
        # LDS banking by each ds_* instruction's lane groups (MI355X LDS table)
        "-gpgpu_shmem_cdna_lane_groups": "1",
        "-gpgpu_shmem_size": "163840",
        "-gpgpu_shmem_sizeDefault": "163840",
        "-gpgpu_shmem_per_block": "163840",
        "-gpgpu_adaptive_cache_config": "0",
        "-gpgpu_unified_l1d_size": "0",
        # vector L1 (TCP): 32 KB, 128 B lines filled whole ('N': a miss fetches
        # every sector of the line it does not hold, like the L2): the 64 B
        # request for the other half of a line the TCP already fetched hits.
        # Against TCP_TCC_READ_REQ over the suite: L1 read misses 3.2 % MAE
        # line-granular vs 26.4 % sectored (profiles/correlation/README.md)
        "-gpgpu_cache:dl1": "N:64:128:4,L:T:m:L:L,A:256:8,16:0,32",
        # instruction cache: 64 KB shared by a CU pair -> 32 KB per CU, modelled
        # (not perfect) because small kernels pay their cold misses
        "-gpgpu_perfect_inst_const_cache": "0",
        # hipMemcpy H2D goes through SDMA to HBM, not through the XCD L2s
        "-gpgpu_perf_sim_memcpy": "0",
        "-gpgpu_cache:il1": "N:64:128:4,L:R:f:N:L,S:8:64,4",
        "-gpgpu_l1_latency": "120",
        "-gpgpu_smem_latency": "64",
        # 4 MiB per XCD (16 x 256 KB), 128 B line fills (TCC_EA0_RDREQ_128B),
        # write-back with byte-masked write allocation ('L')
        "-gpgpu_cache:dl2": "N:128:128:16,L:B:m:L:P,A:192:4,32:0,32",
        # L2 hit = per-XCD L2 (~207 cycles), L2 miss = Infinity Cache (~540)
        "-gpgpu_l2_rop_latency": "75",
        "-dram_latency": "333",
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
        # the CU's scalar unit executes s_* ALU instructions (CDNA traces map
        # them to specialized unit 8)
        "-specialized_unit_8": "1,4,4,4,4,SALU",
        "-trace_opcode_latency_initiation_spec_op_8": "2,1",
        # the SQC instruction cache fetches sequential code lines ahead
        "-gpgpu_inst_prefetch_lines": "8",
        # CDNA4 memory hierarchy: 8 XCDs with private L2s (16 slices each;
        # workgroups round-robin over the XCDs), and the 256 MB Infinity Cache
        # (MALL) as a memory-side cache in front of the 128 HBM channels
        # (2 MB = 1024 sets x 16 ways of 128 B per channel); -dram_latency is
        # the L2-miss path to the MALL (ub_cache_lat: MALL 535 - L2 201
        # cycles), a MALL miss adds the HBM path on top (HBM 889 - MALL 535,
        # less the DRAM timing the channel model adds itself)
        "-sim_xcd": "8",
        "-sim_mall": "1024:16",
        "-sim_mall_miss_latency": "250",
        # the XCD L2s are not coherent with each other: every kernel ends with
        # a release that writes their dirty lines back (to the MALL) and the
        # next one starts with them invalidated
        "-sim_l2_kernel_release": "1",
        # TCP -> TCC writes are at most 64 B (TCC_WRITE counts two requests
        # for a store covering a whole 128 B line)
        "-sim_l1_write_request_bytes": "64",
        # kernel launch as rocprofv3 durations see it (ub_launch +
        # hw_stats/launch_latency.py): 1.5 us from an idle queue to the first
        # workgroup; a kernel queued behind another lasts >= 4.7 us (the
        # command processor's dependent back-to-back dispatch); the run's first
        # kernel pays a cold start; a host loop submits a kernel every ~5-7 us
        # (ub_launch's back-to-back chains).  These are defaults: the tuner
        # replaces every one with the box's own micro-benchmark measurement
        # (hw_stats/launch_latency.py suggest_ lines), none is fitted on the
        # suite
        "-gpgpu_kernel_launch_latency": "3563",
        "-gpgpu_kernel_launch_latency_queued": "3563",
        "-sim_kernel_min_cycles_queued": "11251",
        "-sim_host_launch_interval": "12000",
        "-sim_first_kernel_latency": "5000",
    })
    return c


PRESETS = {
    "GTX480": _gtx480,
    "KEPLER_TITAN": _kepler_titan,
    "TITANX": _titanx,
    "RTX2060_S": _rtx2060_s,
    "QV100": _qv100,
    "GV100": _gv100,
    "TITANV": _titanv,
    "RTX2060": _rtx2060,
    "RTX3070": _rtx3070,
    "MI355X": _mi355x,
}


def get_preset(name: str) -> Dict[str, str]:
    key = name.upper().replace("-SASS", "")
    for pre in ("SM7_", "SM75_", "SM86_", "SM6_", "SM3_", "SM2_"):
        key = key.replace(pre, "")
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
    # -network_mode 1: the Booksim interconnect file next to the configs
    if opts.get("-network_mode", "2").strip() == "1":
        fn = opts.get("-inter_config_file", "").strip()
        spec = _icnt_spec(name_or_opts, fn)
        if spec and not os.path.isabs(fn):
            with open(os.path.join(out_dir, spec[0]), "w") as f:
                f.write(render_icnt(spec[1], f"{spec[0]} ({spec[1]['topology']}, k={spec[1]['k']}, n={spec[1]['n']})"))
    # AccelWattch XMLs next to the configs (SIM / HW / HYBRID modes share the
    # uncalibrated defaults until power.calibrate rewrites them)
    from ..power.xmlcfg import default_params, write_xml
    pname = power_preset or (name_or_opts if isinstance(name_or_opts, str) else "custom")
    for mode in ("sim", "hw", "hybrid"):
        xp = os.path.join(out_dir, f"accelwattch_sass_{mode}.xml")
        if not os.path.exists(xp):
            write_xml(xp, default_params(pname), comment=f"{pname} defaults (uncalibrated)")
    return p1, p2


def _icnt_spec(name_or_opts, fn: str):
    """(file name, params) of the interconnect file a preset / option dict names."""
    if isinstance(name_or_opts, str):
        try:
            key = next(k for k in PRESETS if get_preset(name_or_opts)["-inter_config_file"] == ICNT_FILES.get(k, ("",))[0])
        except (StopIteration, KeyError):
            key = None
        if key in ICNT_FILES:
            return ICNT_FILES[key]
    for f, p in ICNT_FILES.values():
        if f == os.path.basename(fn):
            return f, p
    return None


def _materialise_icnt(opts: Dict[str, str], name_or_opts) -> None:
    """argv use: point -inter_config_file at a generated file in a cache dir."""
    if opts.get("-network_mode", "2").strip() != "1":
        return
    fn = opts.get("-inter_config_file", "").strip()
    if os.path.isabs(fn) or os.path.exists(fn):
        return
    spec = _icnt_spec(name_or_opts, fn)
    if not spec:
        return
    import hashlib
    import tempfile
    text = render_icnt(spec[1], spec[0])
    d = os.path.join(tempfile.gettempdir(), f"asim_icnt_{os.getuid()}")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, hashlib.sha1(text.encode()).hexdigest()[:12] + "_" + spec[0])
    if not os.path.exists(path):
        tmp = path + f".{os.getpid()}"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, path)
    opts["-inter_config_file"] = path


def args_for(name_or_opts, extra: Dict[str, str] | None = None) -> list:
    """Flat argv list (no files) for a preset, for in-process simulators."""
    opts = get_preset(name_or_opts) if isinstance(name_or_opts, str) else dict(name_or_opts)
    if extra:
        opts.update(extra)
    _materialise_icnt(opts, name_or_opts)
    argv = []
    for k, v in opts.items():
        if len(v) >= 2 and v[0] == '"' and v[-1] == '"':
            v = v[1:-1]
        argv += [k, v]
    return argv
