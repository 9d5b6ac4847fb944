#include "sim_options.h"

#include <unistd.h>

#include "icnt_config.h"
#include "../model/addrdec.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <sstream>

namespace asim {

namespace {

struct OptDef {
  const char* name;
  char type;  // b i u I U f s
  const char* deflt;
  const char* help;
};

// Every flag accepted in trace mode.  Defaults follow the documented meaning
// of each flag; values that matter are always set by the tested configs.
const OptDef kOptions[] = {
    // ---- trace frontend ----
    {"-trace", 's', "./traces/kernelslist.g", "traces kernel list file"},
    {"-trace_opcode_latency_initiation_int", 's', "4,1", "int <latency,initiation>"},
    {"-trace_opcode_latency_initiation_sp", 's', "4,1", "sp <latency,initiation>"},
    {"-trace_opcode_latency_initiation_dp", 's', "4,1", "dp <latency,initiation>"},
    {"-trace_opcode_latency_initiation_sfu", 's', "4,1", "sfu <latency,initiation>"},
    {"-trace_opcode_latency_initiation_tensor", 's', "4,1", "tensor <latency,initiation>"},
    // ---- topology / SM ----
    {"-gpgpu_n_clusters", 'u', "10", "number of processing clusters"},
    {"-gpgpu_n_cores_per_cluster", 'u', "3", "SIMT cores per cluster"},
    {"-gpgpu_n_mem", 'u', "8", "number of memory channels"},
    {"-gpgpu_n_sub_partition_per_mchannel", 'u', "1", "L2 sub-partitions per channel"},
    {"-gpgpu_n_mem_per_ctrlr", 'u', "1", "DRAM chips per controller"},
    {"-gpgpu_shader_core_pipeline", 's', "1024:32", "<max threads per SM>:<warp size>"},
    {"-gpgpu_shader_registers", 'u', "8192", "registers per SM"},
    {"-gpgpu_registers_per_block", 'u', "8192", "registers per CTA"},
    {"-gpgpu_ignore_resources_limitation", 'b', "0", "ignore register/shmem limits"},
    {"-gpgpu_shader_cta", 'u', "32", "max CTAs per SM"},
    {"-gpgpu_num_cta_barriers", 'u', "16", "barriers per CTA"},
    {"-gpgpu_n_cluster_ejection_buffer_size", 'u', "8", "cluster ejection buffer"},
    {"-gpgpu_n_ldst_response_buffer_size", 'u', "2", "LD/ST response buffer"},
    {"-gpgpu_shmem_per_block", 'u', "49152", "shared memory per CTA"},
    {"-gpgpu_shmem_size", 'u', "16384", "shared memory per SM"},
    {"-gpgpu_shmem_option", 's', "0", "shared memory carve-out options (KB)"},
    {"-gpgpu_unified_l1d_size", 'u', "0", "unified L1/shmem size (KB)"},
    {"-gpgpu_adaptive_cache_config", 'b', "0", "adaptive L1/shmem split"},
    {"-gpgpu_shmem_sizeDefault", 'u', "16384", "default shmem size"},
    {"-gpgpu_shmem_size_PrefL1", 'u', "16384", "shmem size prefer-L1"},
    {"-gpgpu_shmem_size_PrefShared", 'u', "16384", "shmem size prefer-shared"},
    {"-gpgpu_shmem_num_banks", 'u', "16", "shared memory banks"},
    {"-gpgpu_shmem_limited_broadcast", 'b', "1", "limited broadcast"},
    {"-gpgpu_shmem_cdna_lane_groups", 'b', "0",
     "wave64 traces: bank conflicts per CDNA4 LDS lane group of each ds_* instruction (2 x 32 lanes for b32/b64, "
     "4 x 16 for b128, 8 x 8 for b96 and wide stores; 32 or 64 banks by instruction); the degree is 1 + the extra "
     "cycles (SQ_LDS_BANK_CONFLICT)"},
    {"-gpgpu_shmem_warp_parts", 'i', "2", "warp parts for shmem conflicts"},
    {"-gpgpu_mem_unit_ports", 'i', "1", "memory unit ports"},
    {"-gpgpu_warpdistro_shader", 'i', "-1", "warp distribution shader"},
    {"-gpgpu_warp_issue_shader", 'i', "0", "warp issue shader"},
    {"-gpgpu_local_mem_map", 'b', "1", "local memory mapping"},
    {"-gpgpu_num_reg_banks", 'i', "8", "register file banks"},
    {"-gpgpu_reg_bank_use_warp_id", 'b', "0", "bank index uses warp id"},
    {"-gpgpu_sub_core_model", 'b', "0", "sub-core model"},
    {"-gpgpu_enable_specialized_operand_collector", 'b', "1", "specialized collectors"},
    {"-gpgpu_operand_collector_num_units_sp", 'i', "4", ""},
    {"-gpgpu_operand_collector_num_units_dp", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_units_sfu", 'i', "4", ""},
    {"-gpgpu_operand_collector_num_units_int", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_units_tensor_core", 'i', "4", ""},
    {"-gpgpu_operand_collector_num_units_mem", 'i', "2", ""},
    {"-gpgpu_operand_collector_num_units_gen", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_in_ports_sp", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_in_ports_dp", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_in_ports_sfu", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_in_ports_int", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_in_ports_tensor_core", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_in_ports_mem", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_in_ports_gen", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_out_ports_sp", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_out_ports_dp", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_out_ports_sfu", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_out_ports_int", 'i', "0", ""},
    {"-gpgpu_operand_collector_num_out_ports_tensor_core", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_out_ports_mem", 'i', "1", ""},
    {"-gpgpu_operand_collector_num_out_ports_gen", 'i', "0", ""},
    {"-gpgpu_coalesce_arch", 'i', "13", "coalescing architecture (compute capability)"},
    {"-gpgpu_num_sched_per_core", 'i', "1", "warp schedulers per SM"},
    {"-gpgpu_max_insn_issue_per_warp", 'i', "2", "max instructions issued per warp per cycle"},
    {"-gpgpu_warp_issue_interval", 'u', "1",
     "minimum cycles between two issue cycles of one warp (1 = every cycle; CDNA: the sequencer visits a SIMD's waves every few cycles)"},
    {"-gpgpu_dual_issue_diff_exec_units", 'b', "1", "dual issue to different units only"},
    {"-gpgpu_simt_core_sim_order", 'i', "1", "core simulation order"},
    {"-gpgpu_pipeline_widths", 's', "1,1,1,1,1,1,1,1,1,1,1,1,1", "pipeline register widths"},
    {"-gpgpu_tensor_core_avail", 'u', "0", "tensor cores present"},
    {"-gpgpu_num_sp_units", 'u', "1", ""},
    {"-gpgpu_num_dp_units", 'u', "0", ""},
    {"-gpgpu_num_int_units", 'u', "0", ""},
    {"-gpgpu_num_sfu_units", 'u', "1", ""},
    {"-gpgpu_num_tensor_core_units", 'u', "0", ""},
    {"-gpgpu_num_mem_units", 'u', "1", ""},
    {"-gpgpu_scheduler", 's', "gto", "warp scheduler policy lrr|gto|two_level_active|old|rrr|warp_limiting"},
    {"-gpgpu_concurrent_kernel_sm", 'b', "0", "concurrent kernels per SM"},
    {"-gpgpu_perfect_inst_const_cache", 'b', "0", "perfect instruction/constant cache"},
    {"-gpgpu_inst_fetch_block_bytes", 'u', "0",
     "> 0: a wave's fetch reads the instruction cache once per aligned block of this many bytes it enters (the CDNA "
     "sequencer's instruction buffer holds the block; SQC_ICACHE_HITS + MISSES count these reads); 0: every fetch "
     "probes (GPGPU-Sim)"},
    {"-gpgpu_inst_prefetch_lines", 'u', "0",
     "sequential instruction prefetch: code lines fetched ahead on an L1I miss or on entering a line (0 = off)"},
    {"-gpgpu_inst_fetch_throughput", 'i', "1", "fetch throughput"},
    {"-gpgpu_reg_file_port_throughput", 'i', "1", "register file port throughput"},
    {"-gpgpu_simd_model", 'i', "1", "SIMD model"},
    {"-gpgpu_clock_gated_reg_file", 'b', "0", ""},
    {"-gpgpu_clock_gated_lanes", 'b', "0", ""},
    {"-n_regfile_gating_group", 'u', "4", ""},
    {"-gpgpu_occupancy_sm_number", 'i', "0", "compute capability for occupancy"},
    // ---- caches ----
    {"-gpgpu_cache:dl1", 's', "none", "L1D config"},
    {"-gpgpu_cache:dl1PrefL1", 's', "none", ""},
    {"-gpgpu_cache:dl1PrefShared", 's', "none", ""},
    {"-gpgpu_cache:il1", 's', "N:64:128:16,L:R:f:N:L,S:2:48,4", "L1I config"},
    {"-gpgpu_tex_cache:l1", 's', "N:4:128:256,L:R:m:N:L,T:512:8,128:2", "texture cache"},
    {"-gpgpu_const_cache:l1", 's', "N:128:64:8,L:R:f:N:L,S:2:64,4", "constant cache"},
    {"-gpgpu_l1_cache_write_ratio", 'u', "0", ""},
    {"-gpgpu_l1_banks", 'u', "1", "L1 banks"},
    {"-sim_l1_port_bytes", 'u', "0", "vector L1 data path bytes per cycle (0: off, l1_banks accesses per cycle)"},
    {"-sim_l1_addr_lanes_per_cycle", 'u', "0", "vector L1 address stage lanes per cycle (0: off)"},
    {"-sim_l1_port_granule", 'u', "0",
     "vector L1 data path unit: 32 = whole sectors, 64 = whole 64 B halves of each line an access touches "
     "(0: the bytes the lanes touch)"},
    {"-sim_lds_port_bytes", 'u', "0", "LDS data path bytes per cycle (0: off, the bank-conflict degree only)"},
    {"-sim_lds_lanes_per_cycle", 'u', "0", "LDS address lanes per cycle (0: off)"},
    {"-gpgpu_l1_banks_byte_interleaving", 'u', "32", ""},
    {"-gpgpu_l1_banks_hashing_function", 'u', "0", ""},
    {"-gpgpu_l1_latency", 'u', "1", "L1 hit latency"},
    {"-sim_l1_miss_return_latency", 'u', "0",
     "cycles from an L1 fill (or a bypassing reply) to the load's completion: the vector memory pipeline "
     "a miss traverses besides the L2 round trip (0: none)"},
    {"-gpgpu_smem_latency", 'u', "3", "shared memory latency"},
    {"-gpgpu_gmem_skip_L1D", 'b', "0", "global memory bypasses L1"},
    {"-gpgpu_perfect_mem", 'b', "0", "perfect memory"},
    {"-gpgpu_flush_l1_cache", 'b', "0", "flush L1 between kernels"},
    {"-sim_sqc_invalidate_at_launch", 'b', "0",
     "every kernel launch invalidates the SMs' instruction and scalar-data caches (CDNA's dispatch acquire)"},
    {"-gpgpu_flush_l2_cache", 'b', "0", "flush L2 between kernels"},
    {"-gpgpu_cache:dl2", 's', "64:128:8,L:B:m:N,A:16:4,4", "L2 config"},
    {"-gpgpu_cache:dl2_texture_only", 'b', "1", ""},
    {"-l2_ideal", 'b', "0", ""},
    // ---- memory partition / DRAM ----
    {"-gpgpu_perf_sim_memcpy", 'b', "1", "memcpy fills L2"},
    {"-gpgpu_simple_dram_model", 'b', "0", ""},
    {"-gpgpu_dram_scheduler", 'i', "1", "0 FIFO, 1 FR-FCFS"},
    {"-gpgpu_dram_partition_queues", 's', "8:8:8:8", "icnt->L2:L2->dram:dram->L2:L2->icnt"},
    {"-gpgpu_memlatency_stat", 'i', "0", ""},
    {"-gpgpu_frfcfs_dram_sched_queue_size", 'i', "0", "0 = unlimited"},
    {"-gpgpu_dram_return_queue_size", 'i', "0", "0 = unlimited"},
    {"-gpgpu_dram_buswidth", 'u', "4", "bytes per DRAM bus"},
    {"-gpgpu_dram_burst_length", 'u', "4", ""},
    {"-dram_data_command_freq_ratio", 'u', "2", ""},
    {"-gpgpu_dram_timing_opt", 's', "4:2:8:12:21:13:34:9:4:5:13:1:0:0", "DRAM timing"},
    {"-gpgpu_l2_rop_latency", 'u', "85", "ROP latency"},
    {"-dram_latency", 'u', "30", "DRAM pipeline latency"},
    {"-dram_dual_bus_interface", 'u', "0", ""},
    {"-dram_bnk_indexing_policy", 'u', "0", ""},
    {"-dram_bnkgrp_indexing_policy", 'u', "0", ""},
    {"-dram_seperate_write_queue_enable", 'b', "0", ""},
    {"-dram_write_queue_size", 's', "32:28:16", ""},
    {"-dram_elimnate_rw_turnaround", 'b', "0", ""},
    {"-gpgpu_mem_addr_mapping", 's', "", "dramid@<start bit>;<address map>"},
    {"-gpgpu_mem_addr_test", 'b', "0", "address mapping alias sweep"},
    {"-gpgpu_mem_address_mask", 'i', "0", ""},
    {"-gpgpu_memory_partition_indexing", 'u', "0", "0 none,1 xor,2 ipoly,3 pae,4 random"},
    // ---- interconnect ----
    {"-network_mode", 'i', "2", "1 intersim, 2 local xbar"},
    {"-inter_config_file", 's', "mesh", ""},
    {"-icnt_in_buffer_limit", 'u', "64", ""},
    {"-icnt_out_buffer_limit", 'u', "64", ""},
    {"-icnt_subnets", 'u', "2", ""},
    {"-icnt_arbiter_algo", 'u', "1", ""},
    {"-icnt_verbose", 'u', "0", ""},
    {"-icnt_grant_cycles", 'u', "1", ""},
    {"-icnt_link_contention", 'u', "0", "network_mode 1: 0 off, 1 shared links delay packets (link reservation per epoch), 2 input-queued routers with VCs, credits and the .icnt file's allocator (icnt_router.h)"},
    {"-icnt_flit_size", 'u', "32", "flit size in bytes"},
    // ---- clocks / kernel ----
    {"-gpgpu_clock_domains", 's', "500.0:2000.0:2000.0:2000.0", "core:icnt:L2:DRAM MHz"},
    {"-gpgpu_max_concurrent_kernel", 'i', "32", ""},
    {"-trace_prefetch", 'b', "1", "parse + coalesce the next kernel's trace on a host thread while the engine runs"},
    {"-gpu_ingest", 'b', "1",
     "with -sim_engine gpu: coalesce kernel traces (shared-memory bank conflicts, global line/sector lists) on the MI355X matrix cores"},
    {"-gpu_ingest_min_insts", 'u', "32768",
     "-gpu_ingest: kernels with fewer memory instructions are coalesced on the host (the device round trips cost more)"},
    {"-gpgpu_kernel_launch_latency", 'i', "0", "kernel launch latency (cycles)"},
    {"-gpgpu_kernel_launch_latency_queued", 'i', "-1",
     "launch latency of a kernel queued right behind the previous one (no memcpy / sync between); -1 = as -gpgpu_kernel_launch_latency"},
    {"-gpgpu_TB_launch_latency", 'i', "0", "thread block launch latency"},
    {"-gpgpu_cdp_enabled", 'b', "0", ""},
    {"-gpgpu_max_cycle", 'I', "0", "stop after cycles"},
    {"-gpgpu_max_insn", 'I', "0", "stop after instructions"},
    {"-gpgpu_max_cta", 'i', "0", ""},
    {"-gpgpu_max_completed_cta", 'i', "0", ""},
    {"-gpgpu_runtime_stat", 's', "10000:0", "sample freq:flag"},
    {"-liveness_message_freq", 'I', "1", ""},
    {"-gpgpu_compute_capability_major", 'u', "7", ""},
    {"-gpgpu_compute_capability_minor", 'u', "0", ""},
    {"-gpgpu_deadlock_detect", 'b', "1", "stop on deadlock"},
    {"-gpgpu_stack_size_limit", 'i', "1024", ""},
    {"-gpgpu_heap_size_limit", 'i', "8388608", ""},
    {"-gpgpu_runtime_sync_depth_limit", 'i', "2", ""},
    {"-gpgpu_runtime_pending_launch_count_limit", 'i', "2048", ""},
    {"-gpgpu_cflog_interval", 'i', "0", ""},
    {"-nccl_allreduce_latency", 'i', "100", "constant all-reduce latency (cycles)"},
    // ---- stats / tracing / visualiser ----
    {"-visualizer_enabled", 'b', "0", ""},
    {"-visualizer_outputfile", 's', "", ""},
    {"-visualizer_zlevel", 'i', "6", ""},
    {"-trace_enabled", 'b', "0", "debug trace streams"},
    {"-trace_components", 's', "none", "WARP_SCHEDULER,SCOREBOARD,..."},
    {"-trace_sampling_core", 'i', "0", ""},
    {"-trace_sampling_memory_partition", 'i', "-1", ""},
    {"-enable_ptx_file_line_stats", 'b', "1", ""},
    {"-ptx_line_stats_filename", 's', "gpgpu_inst_stats.txt", ""},
    // ---- PTX-mode flags (accepted, unused in trace mode) ----
    {"-gpgpu_ptx_instruction_classification", 'i', "0", ""},
    {"-gpgpu_ptx_sim_mode", 'i', "0", ""},
    {"-gpgpu_ptx_force_max_capability", 'u', "0", ""},
    {"-gpgpu_ptx_convert_to_ptxplus", 'b', "0", ""},
    {"-gpgpu_ptx_save_converted_ptxplus", 'b', "0", ""},
    {"-gpgpu_ptx_use_cuobjdump", 'b', "1", ""},
    {"-gpgpu_experimental_lib_support", 'b', "0", ""},
    {"-gpgpu_ptx_inst_debug_to_file", 'b', "0", ""},
    {"-gpgpu_ptx_inst_debug_file", 's', "inst_debug.txt", ""},
    {"-gpgpu_ptx_inst_debug_thread_uid", 'i', "1", ""},
    {"-save_embedded_ptx", 'b', "0", ""},
    {"-keep", 'b', "0", ""},
    {"-ptx_opcode_latency_int", 's', "4,13,4,5,145", ""},
    {"-ptx_opcode_latency_fp", 's', "4,13,4,5,39", ""},
    {"-ptx_opcode_latency_dp", 's', "8,19,8,8,330", ""},
    {"-ptx_opcode_latency_sfu", 's', "8", ""},
    {"-ptx_opcode_latency_tesnor", 's', "64", ""},
    {"-ptx_opcode_initiation_int", 's', "1,2,2,2,8", ""},
    {"-ptx_opcode_initiation_fp", 's', "1,2,1,1,4", ""},
    {"-ptx_opcode_initiation_dp", 's', "8,16,8,8,130", ""},
    {"-ptx_opcode_initiation_sfu", 's', "8", ""},
    {"-ptx_opcode_initiation_tensor", 's', "64", ""},
    {"-cdp_latency", 's', "7200,8000,100,12000,1600", ""},
    {"-checkpoint_option", 'i', "0", ""},
    {"-checkpoint_kernel", 'i', "1", ""},
    {"-checkpoint_CTA", 'i', "0", ""},
    {"-resume_option", 'i', "0", ""},
    {"-resume_kernel", 'i', "0", ""},
    {"-resume_CTA", 'i', "0", ""},
    {"-checkpoint_CTA_t", 'i', "0", ""},
    {"-checkpoint_insn_Y", 'i', "0", ""},
    {"-checkpoint_path", 's', "checkpoint_files", "directory of timing-state checkpoints (extension)"},
    // ---- power (AccelWattch) ----
    {"-power_simulation_enabled", 'b', "0", "enable the power model"},
    {"-accelwattch_xml_file", 's', "accelwattch_sass_sim.xml", "power model XML"},
    {"-power_per_cycle_dump", 'b', "0", ""},
    {"-hw_perf_file_name", 's', "hw_perf.csv", ""},
    {"-hw_perf_bench_name", 's', "", ""},
    {"-power_simulation_mode", 'i', "0", "0 SIM, 1 HW, 2 HYBRID"},
    {"-dvfs_enabled", 'b', "0",
     "DVFS governor: with a power_cap in the power XML, run the core below its nominal clock (and voltage) when a "
     "sample's power exceeds the cap; the slower clock lengthens simulated time"},
    {"-dvfs_min_clock_ratio", 'f', "0.5", "lowest core clock / nominal the DVFS governor may choose"},
    {"-aggregate_power_stats", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L1_RH", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L1_RM", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L1_WH", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L1_WM", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L2_RH", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L2_RM", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L2_WH", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_L2_WM", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_CC_ACC", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_SHARED_ACC", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_DRAM_RD", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_DRAM_WR", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_NOC", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_PIPE_DUTY", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_NUM_SM_IDLE", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_CYCLES", 'b', "0", ""},
    {"-accelwattch_hybrid_perfsim_VOLTAGE", 'b', "0", ""},
    {"-power_trace_enabled", 'b', "0", ""},
    {"-power_trace_zlevel", 'i', "6", "(traces are written uncompressed)"},
    {"-power_report_file", 's', "accelwattch_power_report.log", "per-kernel power report (extension)"},
    {"-steady_power_levels_enabled", 'b', "0", ""},
    {"-steady_state_definition", 's', "8:4", ""},
    // ---- legacy / misspelled names used by shipped configs (reference
    // defect D10: these abort the reference; here they are aliases) ----
    {"-gpuwattch_xml_file", 's', "", "legacy alias of -accelwattch_xml_file"},
    {"-smem_latency", 'u', "0", "legacy alias of -gpgpu_smem_latency"},
    {"-gmem_skip_L1D", 'b', "0", "alias of -gpgpu_gmem_skip_L1D"},
    {"-perf_sim_memcpy", 'b', "1", "alias of -gpgpu_perf_sim_memcpy"},
    {"-memory_partition_indexing", 'u', "0", "alias of -gpgpu_memory_partition_indexing"},
    {"-gpgpu_ptx_force_min_capability", 'u', "0", "accepted, unused"},
    // ---- extensions of this simulator ----
    {"-icnt_latency", 'u', "8", "interconnect traversal latency in core cycles (= PDES epoch)"},
    {"-sim_max_outstanding_pkts", 'u', "128", "per-SM packets in flight before injection stalls"},
    {"-sim_engine", 's', "cpu", "cpu | gpu | check (gpu and cpu in lock step, states compared) cycle engine"},
    {"-sim_check_interval", 'u', "4096", "-sim_engine check: cycles between state comparisons"},
    {"-sim_check_primary", 's', "gpu", "-sim_engine check: engine checked against the cpu engine (gpu | cpu)"},
    {"-sim_check_corrupt_at", 'u', "0", "-sim_engine check: perturb the reference state from this cycle (checker self-test)"},
    {"-sim_check_corrupt_mailbox", 'u', "0", "-sim_engine check self-test: perturb a request-mailbox count instead of a unit state"},
    {"-sim_epochs_per_launch", 'u', "4096", "GPU engine epochs per persistent launch"},
    {"-sim_debug", 'b', "0", "interactive timing debugger (reference gpgpu_debug; also GPGPUSIM_DEBUG=1): single step, "
                            "PC / cycle breakpoints, memory-line watchpoints, pipeline dumps"},
    {"-sim_debug_script", 's', "", "debugger commands from this file instead of stdin"},
    {"-sim_debug_step", 'u', "0", "cycles per debugger step (0: one PDES epoch)"},
    {"-sim_break_cycle", 'u', "0", "enter the debugger when the simulation reaches this cycle (reference g_single_step)"},
    {"-collective_model", 's', "const", "const | ring | tree | packet collective timing"},
    {"-xgmi_link_bandwidth_gbps", 'f', "153.0", "per-link xGMI bandwidth (GB/s)"},
    {"-xgmi_link_latency_ns", 'f', "1000.0", "collective step latency (ns)"},
    {"-xgmi_links_per_gpu", 'u', "7", "xGMI links per GPU"},
    {"-sim_event_skip", 'b', "1", "fast-forward quiet SM cycles inside an epoch (results identical)"},
    {"-power_in_loop", 'b', "1",
     "power samples taken by the engine inside its cycle loop (GPU engine: in engine_kernel, f64 MFMA sums), "
     "0 = one engine run per sample with the host evaluating (results identical; DVFS always uses the latter)"},
    {"-trace_host_budget_mb", 'f', "0",
     "read a kernel's text trace per thread block, as the trace window advances, when the file is larger than this "
     "many MiB: host trace memory then follows the window (-gpu_trace_window, 2 when 0) instead of the kernel "
     "(0 = load whole kernels; results identical)"},
    {"-gpu_trace_window", 'i', "4",
     "GPU engine: kernel trace resident in HBM per kernel, in multiples of its resident-CTA capacity; CTAs "
     "stream in as they dispatch (0 = whole kernel; results identical)"},
    {"-sim_xcd", 'u', "0",
     "XCDs with private L2s (0 = one shared L2): SM s belongs to XCD s % N and uses the n_subpart/N slices of its XCD"},
    {"-sim_mall", 's', "none",
     "memory-attached last-level cache (Infinity Cache) per DRAM channel: <sets>:<assoc> of 128 B sectored lines, or none"},
    {"-sim_mall_miss_latency", 'u', "0", "extra core cycles of an HBM access over a MALL hit"},
    {"-sim_host_launch_interval", 'u', "0",
     "host model: core cycles between the host's kernel submissions after a sync (0 = a host that is never the "
     "bottleneck); a kernel submitted after the previous one ended launches into an idle GPU"},
    {"-sim_kernel_min_cycles_queued", 'u', "0",
     "a kernel queued right behind another lasts at least this many core cycles (the command processor's "
     "back-to-back dispatch interval of dependent kernels; 0 = off)"},
    {"-sim_first_kernel_latency", 'u', "0",
     "extra launch cycles of the run's first kernel behind the initial host copies (cold start: the copies' "
     "completion and the first touch of their pages; ub_launch after-copy)"},
    {"-sim_copy_latency_every_kernel", 'b', "0",
     "apply -sim_first_kernel_latency to every kernel launched behind a host copy, not only the run's first "
     "(ub_launch measures it on every one of its copy -> kernel repetitions)"},
    {"-collective_mem_traffic", 'b', "0",
     "run every collective's local memory traffic (send-buffer reads, receive-buffer writes) as an RCCL-style copy "
     "kernel that loads the simulated L2/MALL/HBM and contends with overlapping kernels"},
    {"-sim_l1_write_request_bytes", 'u', "128",
     "largest L1 -> L2 write request: 64 sends a store touching both halves of a line as two requests (gfx950 "
     "TCP -> TCC), 128 one per line"},
    {"-sim_single_valu", 'b', "0",
     "CDNA: integer, fp64 and transcendental vector instructions issue through the SIMD's one VALU (the SP unit of "
     "their scheduler, at their own initiation interval) instead of separate INT / DP / SFU pipelines"},
    {"-sim_l2_kernel_release", 'b', "0",
     "at the end of every kernel write the L2s' dirty sectors back to memory (the MALL if any) and invalidate them "
     "(the release / acquire of a multi-XCD GPU, whose XCD L2s are not coherent with each other)"},
    {"-sim_cpu_threads", 'u', "1", "CPU engine: OpenMP threads over the units of one epoch (1 = serial; "
                                  "run simulations job-parallel instead)"},
    {"-collective_slice_bytes", 'u', "131072", "packet model: bytes per link packet (RCCL slice)"},
    {"-collective_max_channels", 'u', "16", "packet model: max parallel rings (channels)"},
    {"-collective_reduce_gbps", 'f', "900.0", "packet model: local memory bandwidth for reduce/copy (GB/s)"},
};

uint32_t parse_u(const std::string& s, const char* what) {
  char* end = nullptr;
  std::string t = trim(s);
  unsigned long v = strtoul(t.c_str(), &end, 0);
  if (t.empty() || *end) throw OptionError(std::string("bad integer '") + s + "' in " + what);
  return (uint32_t)v;
}

std::pair<uint32_t, uint32_t> parse_lat_ii(const std::string& s, const char* what) {
  auto v = split(strip_ws(s), ',');
  if (v.size() < 2) throw OptionError(std::string("expected <latency,initiation> for ") + what);
  return {parse_u(v[0], what), parse_u(v[1], what)};
}

void mask_limits(uint64_t m, uint8_t& hi, uint8_t& lo) {
  if (!m) {
    hi = 0;
    lo = 0;
    return;
  }
  lo = (uint8_t)__builtin_ctzll(m);
  hi = (uint8_t)(64 - __builtin_clzll(m));
}

uint32_t log2_floor(uint32_t x) {
  uint32_t r = 0;
  while ((1u << (r + 1)) <= x) ++r;
  return r;
}

void setup_addrdec(SimCfg& c, const std::string& mapping, int mask_mode) {
  int chip_s = 10;
  uint64_t m[AF_COUNT] = {0x0000000000001C00ull, 0x0000000000000300ull, 0x000000000FFF0000ull,
                          0x000000000000E0FFull, 0x000000000000000Full};
  switch (mask_mode) {
    case 0:
      chip_s = 10;
      m[AF_CHIP] = 0;
      m[AF_BK] = 0x300;
      m[AF_ROW] = 0x7FFE000;
      m[AF_COL] = 0x1CFF;
      break;
    case 1:
      chip_s = 13;
      m[AF_CHIP] = 0;
      m[AF_BK] = 0x1800;
      m[AF_ROW] = 0x7FFE000;
      m[AF_COL] = 0x7FF;
      break;
    case 2:
    case 3:
      chip_s = 11;
      m[AF_CHIP] = 0;
      m[AF_BK] = 0x1800;
      m[AF_ROW] = mask_mode == 2 ? 0x7FFE000 : 0xFFFE000;
      m[AF_COL] = 0x7FF;
      break;
    default:
      break;
  }
  if (!mapping.empty()) {
    int dramid = -1;
    const char* s = mapping.c_str();
    if (sscanf(s, "dramid@%d", &dramid) == 1) chip_s = dramid;
    else chip_s = -1;
    const char* p = strchr(s, ';');
    p = p ? p + 1 : s;
    for (auto& x : m) x = 0;
    int ofs = 63;
    for (; *p; ++p) {
      switch (*p) {
        case 'D': case 'd':
          if (dramid >= 0) throw OptionError("D bits not allowed together with dramid@");
          m[AF_CHIP] |= 1ull << ofs; --ofs; break;
        case 'B': case 'b': m[AF_BK] |= 1ull << ofs; --ofs; break;
        case 'R': case 'r': m[AF_ROW] |= 1ull << ofs; --ofs; break;
        case 'C': case 'c': m[AF_COL] |= 1ull << ofs; --ofs; break;
        case 'S': case 's': m[AF_BURST] |= 1ull << ofs; m[AF_COL] |= 1ull << ofs; --ofs; break;
        case '0': --ofs; break;
        case '|': case ' ': case '.': break;
        default: throw OptionError(std::string("invalid address mapping character '") + *p + "'");
      }
      if (ofs < -1) break;
    }
    if (ofs != -1) throw OptionError("address mapping must describe exactly 64 bits: " + mapping);
  }
  const uint32_t nch = c.n_mem;
  uint32_t nbits = log2_floor(nch);
  c.log2ch = nbits;
  c.log2sub = log2_floor(c.n_sub_per_mem);
  c.n_ch_pow2 = 1u << nbits;
  c.gap = (nch != (1u << nbits)) ? 1 : 0;
  if (c.gap) {
    nbits++;
    c.n_ch_pow2 <<= 1;
  }
  if (chip_s != -1) {
    if (!c.gap) {
      uint64_t low = (1ull << chip_s) - 1;
      for (int f : {AF_BK, AF_ROW, AF_COL}) m[f] = ((m[f] & ~low) << nbits) | (m[f] & low);
      for (uint32_t i = chip_s; i < chip_s + nbits; ++i) m[AF_CHIP] |= 1ull << i;
    }
  } else if (nch & (nch - 1)) {
    throw OptionError("explicit D-bit address mapping requires a power-of-two channel count");
  }
  if (c.n_sub_per_mem & (c.n_sub_per_mem - 1))
    throw OptionError("sub-partitions per channel must be a power of two");
  c.addr_chip_s = chip_s < 0 ? 0 : chip_s;
  for (int f = 0; f < AF_COUNT; ++f) {
    c.addr_mask[f] = m[f];
    mask_limits(m[f], c.mk_hi[f], c.mk_lo[f]);
  }
  c.sub_id_mask = 0;
  if (c.n_sub_per_mem > 1) {
    uint32_t need = c.log2sub, pos = 0;
    for (int i = c.mk_lo[AF_BK]; i < c.mk_hi[AF_BK] && pos < need; ++i)
      if (m[AF_BK] >> i & 1ull) {
        c.sub_id_mask |= 1ull << i;
        ++pos;
      }
  }
  for (int f = 0; f < AF_COUNT; ++f) c.addr_runs[f] = make_runs(c.addr_mask[f], c.mk_hi[f], c.mk_lo[f]);
  c.part_runs = make_runs(c.gap ? ~c.sub_id_mask : ~(c.addr_mask[AF_CHIP] | c.sub_id_mask), 64, 0);
}

void parse_dram_timing(SimCfg& c, const std::string& s0) {
  std::string s = strip_ws(s0);
  if (s.find('=') != std::string::npos) {
    for (auto& kv : split(s, ':')) {
      if (kv.empty()) continue;
      auto eq = kv.find('=');
      if (eq == std::string::npos) throw OptionError("bad DRAM timing token '" + kv + "'");
      std::string k = kv.substr(0, eq);
      uint32_t v = parse_u(kv.substr(eq + 1), "-gpgpu_dram_timing_opt");
      if (k == "nbk") c.nbk = v;
      else if (k == "CCD") c.tCCD = v;
      else if (k == "RRD") c.tRRD = v;
      else if (k == "RCD") c.tRCD = v;
      else if (k == "RAS") c.tRAS = v;
      else if (k == "RP") c.tRP = v;
      else if (k == "RC") c.tRC = v;
      else if (k == "CL") c.CL = v;
      else if (k == "WL") c.WL = v;
      else if (k == "CDLR") c.tCDLR = v;
      else if (k == "WR") c.tWR = v;
      else if (k == "nbkgrp") c.nbkgrp = v;
      else if (k == "CCDL") c.tCCDL = v;
      else if (k == "RTPL") c.tRTPL = v;
      else throw OptionError("unknown DRAM timing parameter '" + k + "'");
    }
  } else {
    auto v = split(s, ':');
    uint32_t* dst[] = {&c.nbk, &c.tCCD, &c.tRRD, &c.tRCD, &c.tRAS, &c.tRP, &c.tRC,
                       &c.CL,  &c.WL,   &c.tCDLR, &c.tWR, &c.nbkgrp, &c.tCCDL, &c.tRTPL};
    for (size_t i = 0; i < v.size() && i < 14; ++i) *dst[i] = parse_u(v[i], "-gpgpu_dram_timing_opt");
  }
  if (!c.nbkgrp) c.nbkgrp = 1;
  if (c.nbk > (uint32_t)kMaxBanksDram) throw OptionError("too many DRAM banks for this build");
}

uint8_t sched_of(const std::string& s) {
  if (s.rfind("lrr", 0) == 0) return SCHED_LRR;
  if (s.rfind("gto", 0) == 0) return SCHED_GTO;
  if (s.rfind("old", 0) == 0) return SCHED_OLDEST;
  if (s.rfind("rrr", 0) == 0) return SCHED_RRR;
  if (s.rfind("two_level_active", 0) == 0) return SCHED_TWO_LEVEL;
  if (s.rfind("warp_limiting", 0) == 0) return SCHED_WARP_LIMITING;
  throw OptionError("unknown scheduler '" + s + "'");
}

}  // namespace

void register_sim_options(OptionRegistry& r) {
  for (const auto& d : kOptions) {
    OptType t;
    switch (d.type) {
      case 'b': t = OptType::Bool; break;
      case 'i': t = OptType::Int32; break;
      case 'u': t = OptType::UInt32; break;
      case 'I': t = OptType::Int64; break;
      case 'U': t = OptType::UInt64; break;
      case 'f': t = OptType::Double; break;
      default: t = OptType::Str; break;
    }
    r.reg(d.name, t, d.help, d.deflt);
  }
  for (int j = 1; j <= 8; ++j) {
    r.reg("-specialized_unit_" + std::to_string(j), OptType::Str,
          "<enabled>,<num_units>,<max_latency>,<ID_OC_SPEC>,<OC_EX_SPEC>,<NAME>", "0,4,4,4,4,BRA");
    r.reg("-trace_opcode_latency_initiation_spec_op_" + std::to_string(j), OptType::Str,
          "specialized unit <latency,initiation>", "4,4");
  }
}

CacheGeom parse_cache_geom(const std::string& s0, bool any_line) {
  CacheGeom g{};
  std::string s = strip_ws(s0);
  if (s == "none" || s.empty()) {
    g.disabled = 1;
    g.nsets = 1;
    g.assoc = 1;
    g.line = 128;
    g.mshr_entries = 1;
    g.mshr_merge = 1;
    return g;
  }
  char ct, rp, wp, ap, mt, wap = 'N', sif = 'L';
  unsigned nset, line, assoc, mshr = 0, merge = 0, mq = 0, rfe = 0, dpw = 0;
  int n = sscanf(s.c_str(), "%c:%u:%u:%u,%c:%c:%c:%c:%c,%c:%u:%u,%u:%u,%u", &ct, &nset, &line, &assoc, &rp, &wp, &ap,
                 &wap, &sif, &mt, &mshr, &merge, &mq, &rfe, &dpw);
  if (n < 12) {
    // older 4-field policy section: <rep>:<wr>:<alloc>:<wr_alloc>
    n = sscanf(s.c_str(), "%c:%u:%u:%u,%c:%c:%c:%c,%c:%u:%u,%u", &ct, &nset, &line, &assoc, &rp, &wp, &ap, &wap, &mt,
               &mshr, &merge, &mq);
    sif = 'L';
    if (n < 11) {
      // oldest form without sector flag: <sets>:<line>:<assoc>,...
      ct = 'N';
      n = sscanf(s.c_str(), "%u:%u:%u,%c:%c:%c:%c,%c:%u:%u,%u", &nset, &line, &assoc, &rp, &wp, &ap, &wap, &mt, &mshr,
                 &merge, &mq);
      if (n < 10) throw OptionError("cannot parse cache config '" + s0 + "'");
    }
  }
  if (ct != 'N' && ct != 'S') throw OptionError("cache type must be N or S: " + s0);
  g.sectored = ct == 'S';
  g.nsets = nset;
  g.line = line;
  g.assoc = assoc;
  g.repl = rp == 'F' ? REPL_FIFO : REPL_LRU;
  switch (wp) {
    case 'R': g.wpolicy = WP_READ_ONLY; break;
    case 'B': g.wpolicy = WP_WRITE_BACK; break;
    case 'T': g.wpolicy = WP_WRITE_THROUGH; break;
    case 'E': g.wpolicy = WP_WRITE_EVICT; break;
    case 'L': g.wpolicy = WP_LOCAL_WB_GLOBAL_WT; break;
    default: throw OptionError("bad cache write policy in " + s0);
  }
  g.alloc = (uint8_t)ap;
  g.walloc = (uint8_t)wap;
  switch (sif) {
    case 'H': g.set_index = SIDX_FERMI; break;
    case 'P': g.set_index = SIDX_HASH_IPOLY; break;
    case 'X': g.set_index = SIDX_BITWISE_XOR; break;
    case 'C': g.set_index = SIDX_CUSTOM; break;
    default: g.set_index = SIDX_LINEAR; break;
  }
  g.mshr_entries = mshr ? mshr : 1;
  g.mshr_merge = merge ? merge : 1;
  g.miss_queue = mq;
  if (any_line && g.line != 128 && g.line >= 16 && g.line <= 128 && !(g.line & (g.line - 1))) {
    // read-only caches of smaller lines: same capacity in 128 B lines
    g.nsets = std::max<uint32_t>(1, g.nsets * g.line / 128);
    g.line = 128;
  }
  if (g.line != 128) throw OptionError("only 128-byte cache lines are supported: " + s0);
  if (g.nsets & (g.nsets - 1)) throw OptionError("cache set count must be a power of two: " + s0);
  return g;
}

// a relative file named by an option: as given if readable, else next to the
// -config files (most recent first), like a run directory's copies
static std::string resolve_cfg_path(const OptionRegistry& r, const std::string& f) {
  auto exists = [](const std::string& p) { return access(p.c_str(), R_OK) == 0; };
  if (f.empty() || f[0] == '/' || exists(f)) return f;
  const auto& dirs = r.config_dirs();
  for (auto it = dirs.rbegin(); it != dirs.rend(); ++it)
    if (exists(*it + "/" + f)) return *it + "/" + f;
  return f;
}

namespace {
// why an accepted option has no effect here
struct Unmodelled {
  const char* name;  // exact name, or a prefix ending in '*'
  const char* why;
  const char* same;  // a value that leaves the modelled behaviour unchanged (no message), or null
};
const char* const kPtxOnly = "PTX (execution-driven) mode only; this is a trace-driven simulator";
const char* const kNotModelled = "accepted for config compatibility, not modelled";
const char* const kPtxLat = "PTX-mode latencies; trace mode times instructions with -trace_opcode_latency_initiation_*";
const char* const kCoalesce = "the trace-ingest coalescer always applies the sectored (sm_70+) rules";
const Unmodelled kUnmodelled[] = {
    {"-gpgpu_ptx_*", kPtxOnly}, {"-save_embedded_ptx", kPtxOnly}, {"-keep", kPtxOnly},
    {"-enable_ptx_file_line_stats", kPtxOnly}, {"-ptx_line_stats_filename", kPtxOnly},
    {"-gpgpu_experimental_lib_support", kPtxOnly}, {"-gpgpu_cdp_enabled", kPtxOnly}, {"-cdp_latency", kPtxOnly},
    {"-gpgpu_compute_capability_major", kPtxOnly}, {"-gpgpu_compute_capability_minor", kPtxOnly},
    {"-gpgpu_stack_size_limit", kPtxOnly}, {"-gpgpu_heap_size_limit", kPtxOnly},
    {"-gpgpu_runtime_sync_depth_limit", kPtxOnly}, {"-gpgpu_runtime_pending_launch_count_limit", kPtxOnly},
    {"-checkpoint_CTA", kPtxOnly}, {"-resume_CTA", kPtxOnly}, {"-checkpoint_CTA_t", kPtxOnly},
    {"-checkpoint_insn_Y", kPtxOnly}, {"-gpgpu_occupancy_sm_number", kPtxOnly},
    {"-ptx_opcode_latency_*", kPtxLat}, {"-ptx_opcode_initiation_*", kPtxLat},
    {"-gpgpu_coalesce_arch", kCoalesce},
    {"-gpgpu_simd_model", kNotModelled},
    {"-gpgpu_reg_bank_use_warp_id", "the reference ignores it too: register banks always include the warp id (shader.cc:4141-4144)"},
    {"-gpgpu_mem_unit_ports", kNotModelled}, {"-gpgpu_num_mem_units", "one LD/ST unit per SM"},
    {"-gpgpu_operand_collector_num_in_ports_*", "collector ports are not a separate resource here"},
    {"-gpgpu_operand_collector_num_out_ports_*", "collector ports are not a separate resource here"},
    {"-gpgpu_tex_cache:l1", "texture path not modelled (no texture instructions in CDNA traces)"},
    {"-gpgpu_const_cache:l1", "constant loads go through the L1D / scalar-cache path"},
    {"-gpgpu_l1_banks_byte_interleaving", kNotModelled}, {"-gpgpu_l1_banks_hashing_function", kNotModelled},
    {"-gpgpu_cache:dl2_texture_only", kNotModelled, "0"}, {"-l2_ideal", kNotModelled},
    {"-icnt_out_buffer_limit", kNotModelled}, {"-icnt_subnets", "the crossbar always has separate request / reply subnets"},
    {"-icnt_verbose", kNotModelled}, {"-gpgpu_clock_gated_reg_file", kNotModelled},
    {"-gpgpu_clock_gated_lanes", kNotModelled}, {"-n_regfile_gating_group", kNotModelled},
    {"-gpgpu_registers_per_block", kPtxOnly}, {"-gpgpu_ignore_resources_limitation", kNotModelled},
    {"-gpgpu_num_cta_barriers", kNotModelled}, {"-gpgpu_shmem_sizeDefault", kNotModelled},
    {"-gpgpu_shmem_size_PrefL1", kNotModelled}, {"-gpgpu_shmem_size_PrefShared", kNotModelled},
    {"-gpgpu_cache:dl1PrefL1", kNotModelled}, {"-gpgpu_cache:dl1PrefShared", kNotModelled},
    {"-gpgpu_warpdistro_shader", kNotModelled}, {"-gpgpu_warp_issue_shader", kNotModelled},
    {"-gpgpu_local_mem_map", kNotModelled}, {"-gpgpu_simt_core_sim_order", kNotModelled},
    {"-power_per_cycle_dump", kNotModelled}, {"-aggregate_power_stats", kNotModelled},
    {"-power_trace_zlevel", kNotModelled}, {"-visualizer_zlevel", kNotModelled}, {"-gpgpu_cflog_interval", kNotModelled},
    {"-liveness_message_freq", kNotModelled}, {"-gpgpu_mem_addr_test", kNotModelled},
};
bool unmodelled_match(const char* pat, const std::string& name) {
  const size_t n = strlen(pat);
  if (n && pat[n - 1] == '*') return name.compare(0, n - 1, pat, n - 1) == 0;
  return name == pat;
}
}  // namespace

std::vector<std::string> unmodelled_option_warnings(const OptionRegistry& r) {
  std::vector<std::string> out;
  for (const auto& kv : r.user_values()) {
    const OptionRegistry::Opt* o = r.find(kv.first);
    if (!o || o->value == o->deflt) continue;
    // the default carve-out only differs from -gpgpu_shmem_size when set apart
    if (kv.first == "-gpgpu_shmem_sizeDefault" && r.getu(kv.first) == r.getu("-gpgpu_shmem_size")) continue;
    for (const Unmodelled& u : kUnmodelled)
      if (unmodelled_match(u.name, kv.first)) {
        if (u.same && kv.second == u.same) break;
        const bool note = u.why == kPtxOnly || u.why == kPtxLat || u.why == kCoalesce;
        out.push_back(std::string(note ? "note: option " : "WARNING option ") + kv.first + " " + kv.second + ": " +
                      u.why);
        break;
      }
  }
  return out;
}

SimCfg derive_sim_cfg(const OptionRegistry& r) {
  SimCfg c;
  memset(&c, 0, sizeof(c));
  c.n_clusters = (uint32_t)r.getu("-gpgpu_n_clusters");
  c.cores_per_cluster = (uint32_t)r.getu("-gpgpu_n_cores_per_cluster");
  c.n_sm = c.n_clusters * c.cores_per_cluster;
  c.n_mem = (uint32_t)r.getu("-gpgpu_n_mem");
  c.n_sub_per_mem = (uint32_t)r.getu("-gpgpu_n_sub_partition_per_mchannel");
  c.n_subpart = c.n_mem * c.n_sub_per_mem;
  if (c.n_sm == 0 || c.n_sm > (uint32_t)kMaxSmTot) throw OptionError("SM count out of range (1..512)");
  if (c.n_mem == 0 || c.n_mem > (uint32_t)kMaxSubTot) throw OptionError("channel count out of range");
  if (c.n_sub_per_mem > (uint32_t)kMaxSubPerCh) throw OptionError("at most 2 sub-partitions per channel");
  if (c.n_subpart > (uint32_t)kMaxSubTot) throw OptionError("too many L2 sub-partitions");
  {
    auto v = split(strip_ws(r.gets("-gpgpu_shader_core_pipeline")), ':');
    if (v.size() < 2) throw OptionError("-gpgpu_shader_core_pipeline expects <threads>:<warp size>");
    c.max_threads_per_sm = parse_u(v[0], "pipeline");
    c.warp_size = parse_u(v[1], "pipeline");
    if (c.warp_size != 32 && c.warp_size != 64) throw OptionError("warp size must be 32 or 64");
    c.max_warps_per_sm = c.max_threads_per_sm / c.warp_size;
    if (c.max_warps_per_sm > (uint32_t)kMaxWarps) throw OptionError("more than 64 warps per SM");
  }
  c.max_cta_per_sm = std::min<uint32_t>((uint32_t)r.getu("-gpgpu_shader_cta"), kMaxCta);
  c.concurrent_kernel_sm = r.getb("-gpgpu_concurrent_kernel_sm") ? 1u : 0u;
  c.max_concurrent_kernel =
      (uint32_t)std::max<long long>(1, std::min<long long>(kMaxConc, r.geti("-gpgpu_max_concurrent_kernel")));
  c.regs_per_sm = (uint32_t)r.getu("-gpgpu_shader_registers");
  c.shmem_per_sm = (uint32_t)r.getu("-gpgpu_shmem_size");
  c.shmem_per_block = (uint32_t)r.getu("-gpgpu_shmem_per_block");
  c.n_sched = (uint32_t)std::max<long long>(1, r.geti("-gpgpu_num_sched_per_core"));
  if (c.n_sched > (uint32_t)kMaxSched) throw OptionError("at most 4 schedulers per SM");
  for (uint32_t sc = 0; sc < (uint32_t)kMaxSched; ++sc) {
    c.sched_mask[sc] = 0;
    for (uint32_t w = sc; w < c.max_warps_per_sm && sc < c.n_sched; w += c.n_sched) c.sched_mask[sc] |= 1ull << w;
  }
  c.sched_policy = sched_of(r.gets("-gpgpu_scheduler"));
  c.sub_core = r.getb("-gpgpu_sub_core_model") ? 1 : 0;
  c.fetch_throughput = (uint32_t)std::max<long long>(1, r.geti("-gpgpu_inst_fetch_throughput"));
  c.max_issue_per_warp = (uint32_t)std::max<long long>(1, r.geti("-gpgpu_max_insn_issue_per_warp"));
  c.warp_issue_interval = std::max<uint32_t>(1, (uint32_t)r.getu("-gpgpu_warp_issue_interval"));
  c.dual_issue_diff = r.getb("-gpgpu_dual_issue_diff_exec_units") ? 1u : 0u;
  {
    // scheduler parameters: two_level_active:<max_active>:<inner>:<outer>,
    // warp_limiting:<prioritization>:<warps to limit>
    const std::string sp = r.gets("-gpgpu_scheduler");
    const auto f = split(sp, ':');
    c.sched_param = 0;
    if (c.sched_policy == SCHED_TWO_LEVEL) c.sched_param = f.size() > 1 ? parse_u(f[1], "-gpgpu_scheduler") : 6;
    if (c.sched_policy == SCHED_WARP_LIMITING) {
      if (f.size() < 3) throw OptionError("warp_limiting needs warp_limiting:<prio>:<warps>");
      c.sched_param = parse_u(f[2], "-gpgpu_scheduler");
    }
    if ((c.sched_policy == SCHED_TWO_LEVEL || c.sched_policy == SCHED_WARP_LIMITING) && c.sched_param == 0)
      throw OptionError("scheduler limit must be >= 1: " + sp);
  }
  // execution units
  c.unit_count[U_SP] = (uint32_t)r.getu("-gpgpu_num_sp_units");
  c.unit_count[U_DP] = (uint32_t)r.getu("-gpgpu_num_dp_units");
  c.unit_count[U_INT] = (uint32_t)r.getu("-gpgpu_num_int_units");
  c.unit_count[U_SFU] = (uint32_t)r.getu("-gpgpu_num_sfu_units");
  c.unit_count[U_TENSOR] = r.getu("-gpgpu_tensor_core_avail") ? (uint32_t)r.getu("-gpgpu_num_tensor_core_units") : 0;
  c.unit_count[U_MEM] = 1;
  for (int j = 0; j < 8; ++j) {
    auto f = split(strip_ws(r.gets("-specialized_unit_" + std::to_string(j + 1))), ',');
    if (f.size() >= 2 && parse_u(f[0], "specialized_unit") != 0)
      c.unit_count[U_SPEC1 + j] = parse_u(f[1], "specialized_unit");
  }
  {
    auto w = split(strip_ws(r.gets("-gpgpu_pipeline_widths")), ',');
    c.ex_wb_width = w.size() > 10 ? parse_u(w[10], "pipeline widths") : 1;
    if (c.ex_wb_width == 0) c.ex_wb_width = 1;
    for (int u = 0; u < U_COUNT; ++u) c.id_oc_width[u] = c.n_sched;
  }
  // trace-mode latencies per op class
  for (int k = 0; k < OC_COUNT; ++k) {
    c.lat[k] = 1;
    c.ii[k] = 1;
  }
  auto set_li = [&](const char* opt, std::initializer_list<int> classes) {
    auto li = parse_lat_ii(r.gets(opt), opt);
    if (li.first >= (uint32_t)kWbRing) throw OptionError(std::string("latency too large in ") + opt);
    for (int k : classes) {
      c.lat[k] = (uint16_t)li.first;
      c.ii[k] = (uint16_t)std::max<uint32_t>(1, li.second);
    }
  };
  set_li("-trace_opcode_latency_initiation_int", {OC_ALU, OC_INTP, OC_BRANCH});
  set_li("-trace_opcode_latency_initiation_sp", {OC_SP});
  set_li("-trace_opcode_latency_initiation_dp", {OC_DP});
  set_li("-trace_opcode_latency_initiation_sfu", {OC_SFU});
  set_li("-trace_opcode_latency_initiation_tensor", {OC_TENSOR});
  for (int j = 0; j < 8; ++j) {
    std::string n = "-trace_opcode_latency_initiation_spec_op_" + std::to_string(j + 1);
    set_li(n.c_str(), {OC_SPEC1 + j});
  }
  // operand collectors
  if (r.getb("-gpgpu_enable_specialized_operand_collector")) {
    long long n = r.geti("-gpgpu_operand_collector_num_units_sp") + r.geti("-gpgpu_operand_collector_num_units_dp") +
                  r.geti("-gpgpu_operand_collector_num_units_sfu") + r.geti("-gpgpu_operand_collector_num_units_int") +
                  r.geti("-gpgpu_operand_collector_num_units_tensor_core") +
                  r.geti("-gpgpu_operand_collector_num_units_mem") + r.geti("-gpgpu_operand_collector_num_units_gen");
    c.oc_units = (uint32_t)std::max<long long>(1, n);
  } else {
    c.oc_units = (uint32_t)std::max<long long>(1, r.geti("-gpgpu_operand_collector_num_units_gen"));
  }
  c.oc_units = std::min<uint32_t>(c.oc_units, kMaxOC);
  c.reg_banks = (uint32_t)std::max<long long>(1, r.geti("-gpgpu_num_reg_banks"));
  if (c.reg_banks > (uint32_t)kMaxBanks) throw OptionError("too many register banks");
  c.reg_port_tp = (uint32_t)std::max<long long>(1, r.geti("-gpgpu_reg_file_port_throughput"));
  // LD/ST
  c.smem_banks = (uint32_t)r.getu("-gpgpu_shmem_num_banks");
  auto user_set = [&](const char* n) {
    const OptionRegistry::Opt* o = r.find(n);
    return o && o->parsed;
  };
  c.smem_latency = (uint32_t)r.getu(user_set("-smem_latency") ? "-smem_latency" : "-gpgpu_smem_latency");
  c.smem_warp_parts = (uint32_t)std::max<long long>(1, r.geti("-gpgpu_shmem_warp_parts"));
  c.smem_limited_bcast = r.getb("-gpgpu_shmem_limited_broadcast") ? 1 : 0;
  c.smem_cdna_groups = r.getb("-gpgpu_shmem_cdna_lane_groups") ? 1 : 0;
  c.l1 = parse_cache_geom(r.gets("-gpgpu_cache:dl1"));
  c.l1_latency = (uint32_t)r.getu("-gpgpu_l1_latency");
  c.l1_miss_ret = (uint32_t)r.getu("-sim_l1_miss_return_latency");
  if (c.l1_miss_ret + 16 >= (uint32_t)kHitRing) throw OptionError("-sim_l1_miss_return_latency too large");
  c.l1_banks = std::max<uint32_t>(1, (uint32_t)r.getu("-gpgpu_l1_banks"));
  c.l1_port_bytes = (uint32_t)r.getu("-sim_l1_port_bytes");
  c.l1_addr_lanes = (uint32_t)r.getu("-sim_l1_addr_lanes_per_cycle");
  c.l1_port_granule = (uint32_t)r.getu("-sim_l1_port_granule");
  if (c.l1_port_granule && c.l1_port_granule != 32 && c.l1_port_granule != 64)
    throw OptionError("-sim_l1_port_granule must be 0, 32 or 64");
  c.lds_port_bytes = (uint32_t)r.getu("-sim_lds_port_bytes");
  c.lds_lanes = (uint32_t)r.getu("-sim_lds_lanes_per_cycle");
  c.gmem_skip_l1 = r.getb(user_set("-gmem_skip_L1D") ? "-gmem_skip_L1D" : "-gpgpu_gmem_skip_L1D") ? 1 : 0;
  c.adaptive_l1 = r.getb("-gpgpu_adaptive_cache_config") ? 1 : 0;
  c.unified_l1_kb = (uint32_t)r.getu("-gpgpu_unified_l1d_size");
  c.l1_write_ratio = (uint32_t)r.getu("-gpgpu_l1_cache_write_ratio");
  c.perfect_icache = r.getb("-gpgpu_perfect_inst_const_cache") ? 1u : 0u;
  {
    const uint64_t fb = r.getu("-gpgpu_inst_fetch_block_bytes");
    if (fb && (fb & (fb - 1))) throw OptionError("-gpgpu_inst_fetch_block_bytes must be a power of two");
    c.ifetch_block = (uint32_t)std::min<uint64_t>(fb, 128);
  }
  c.inst_prefetch = (uint32_t)std::min<uint64_t>(r.getu("-gpgpu_inst_prefetch_lines"), kMaxIL1Mshr);
  c.il1 = parse_cache_geom(r.gets("-gpgpu_cache:il1"), true);
  if (!c.il1.disabled) {
    // the tag array lives in LDS next to the SM state: keep the associativity,
    // cap the set count (kernels' code rarely exceeds 64 KB)
    while ((uint64_t)c.il1.nsets * c.il1.assoc > (uint64_t)kMaxIL1Lines && c.il1.nsets > 1) c.il1.nsets >>= 1;
    if ((uint64_t)c.il1.nsets * c.il1.assoc > (uint64_t)kMaxIL1Lines) c.il1.assoc = kMaxIL1Lines;
    c.il1.mshr_entries = std::min<uint32_t>(std::max<uint32_t>(1, c.il1.mshr_entries), kMaxIL1Mshr);
  }
  {
    auto v = split(strip_ws(r.gets("-gpgpu_shmem_option")), ',');
    for (auto& x : v) {
      if (x.empty() || c.n_shmem_opts >= 8) continue;
      c.shmem_opts_kb[c.n_shmem_opts++] = parse_u(x, "-gpgpu_shmem_option");
    }
    std::sort(c.shmem_opts_kb, c.shmem_opts_kb + c.n_shmem_opts);
  }
  if (c.l1_latency + 2 >= (uint32_t)kHitRing || c.smem_latency + 34 >= (uint32_t)kHitRing)
    throw OptionError("L1 / shared-memory latency exceeds the completion ring");
  if (!c.l1.disabled && (uint64_t)c.l1.nsets * c.l1.assoc > (uint64_t)kMaxL1Lines)
    throw OptionError("L1 larger than 1024 lines is not supported in this build");
  c.l1.mshr_entries = std::min<uint32_t>(c.l1.mshr_entries, kMaxL1Mshr);
  // interconnect
  c.icnt_latency = (uint32_t)r.getu("-icnt_latency");
  if (c.icnt_latency < 1 || c.icnt_latency > (uint32_t)kMaxEpoch)
    throw OptionError("-icnt_latency must be in 1.." + std::to_string(kMaxEpoch) + " (epoch length)");
  c.flit_size = std::max<uint32_t>(8, (uint32_t)r.getu("-icnt_flit_size"));
  c.icnt_arbiter = r.getu("-icnt_arbiter_algo") ? 1u : 0u;
  c.icnt_grant_cycles = std::max<uint32_t>(1, (uint32_t)r.getu("-icnt_grant_cycles"));
  {
    // the injection buffer holds -icnt_in_buffer_limit flits; a packet is at
    // most a 128-byte line plus its header (reference mem_fetch sizes)
    const uint32_t max_flits = (136 + c.flit_size - 1) / c.flit_size;
    c.icnt_in_pkts = std::max<uint32_t>(1, std::min<uint32_t>(kOutQ, (uint32_t)r.getu("-icnt_in_buffer_limit") / max_flits));
  }
  c.icnt_out_limit = std::min<uint32_t>((uint32_t)r.getu("-sim_max_outstanding_pkts"), kInQ);
  if (c.icnt_out_limit == 0) c.icnt_out_limit = 1;
  c.eject_buf = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)r.getu("-gpgpu_n_cluster_ejection_buffer_size"), kEjectQ));
  c.ldst_resp_buf = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)r.getu("-gpgpu_n_ldst_response_buffer_size"), kLdstRespQ));
  // memory partition
  c.l2 = parse_cache_geom(r.gets("-gpgpu_cache:dl2"));
  if (!c.l2.disabled && (uint64_t)c.l2.nsets * c.l2.assoc * std::max<uint32_t>(1, c.n_sub_per_mem) >
                            (uint64_t)kMaxL2LinesCh)
    throw OptionError("L2 lines per memory channel (sets x assoc x sub-partitions) above " +
                      std::to_string(kMaxL2LinesCh) + " are not supported in this build");
  c.l2.mshr_entries = std::min<uint32_t>(c.l2.mshr_entries, kMaxL2Mshr);
  c.rop_latency = (uint32_t)r.getu("-gpgpu_l2_rop_latency");
  c.dram_latency = (uint32_t)r.getu("-dram_latency");
  {
    auto q = split(strip_ws(r.gets("-gpgpu_dram_partition_queues")), ':');
    uint32_t v[4] = {8, 8, 8, 8};
    for (size_t i = 0; i < q.size() && i < 4; ++i) v[i] = parse_u(q[i], "-gpgpu_dram_partition_queues");
    c.q_icnt_l2 = std::max<uint32_t>(1, v[0]);
    c.q_l2_dram = std::max<uint32_t>(4, v[1]);
    c.q_dram_l2 = std::max<uint32_t>(1, std::min<uint32_t>(v[2], 64));
    c.q_l2_icnt = std::max<uint32_t>(1, v[3]);
  }
  c.perf_memcpy = r.getb(user_set("-perf_sim_memcpy") ? "-perf_sim_memcpy" : "-gpgpu_perf_sim_memcpy") ? 1 : 0;
  // DRAM
  c.dram_sched = (uint32_t)r.geti("-gpgpu_dram_scheduler") ? 1 : 0;
  {
    long long q = r.geti("-gpgpu_frfcfs_dram_sched_queue_size");
    c.dram_queue = (q <= 0 || q > kDramQ) ? (uint32_t)kDramQ : (uint32_t)q;
    long long rq = r.geti("-gpgpu_dram_return_queue_size");
    c.dram_ret_queue = (rq <= 0 || rq > kDramRet) ? (uint32_t)kDramRet : (uint32_t)rq;
  }
  {
    // shared credit pool of the reference's L2->DRAM arbitration: scheduler
    // queue + return queue (0 = unlimited -> the pipe size)
    long long q = r.geti("-gpgpu_frfcfs_dram_sched_queue_size"), rq = r.geti("-gpgpu_dram_return_queue_size");
    uint64_t cr = (q <= 0 || rq <= 0) ? (uint64_t)kDramLat : (uint64_t)q + (uint64_t)rq;
    c.dram_credits = (uint32_t)std::min<uint64_t>(cr, kDramLat);
    // the per-sub-partition L2->DRAM queue plus its share of the pool
    c.q_l2_dram = std::min<uint32_t>(c.q_l2_dram + c.dram_credits / std::max<uint32_t>(1, c.n_sub_per_mem), kDramLat);
  }
  parse_dram_timing(c, r.gets("-gpgpu_dram_timing_opt"));
  c.rw_turnaround = r.getb("-dram_elimnate_rw_turnaround") ? 0u : 1u;
  c.wq_enable = r.getb("-dram_seperate_write_queue_enable") ? 1u : 0u;
  {
    auto v = split(strip_ws(r.gets("-dram_write_queue_size")), ':');
    if (v.size() != 3) throw OptionError("-dram_write_queue_size expects <size>:<high>:<low>");
    c.wq_size = parse_u(v[0], "-dram_write_queue_size");
    c.wq_hi = parse_u(v[1], "-dram_write_queue_size");
    c.wq_lo = parse_u(v[2], "-dram_write_queue_size");
    if (c.wq_enable) {
      // reads and writes share the kDramQ-entry pool
      c.wq_size = std::max<uint32_t>(1, std::min<uint32_t>(c.wq_size, kDramQ / 2));
      c.dram_queue = std::min<uint32_t>(c.dram_queue, (uint32_t)kDramQ - c.wq_size);
      c.wq_hi = std::min(c.wq_hi, c.wq_size);
      c.wq_lo = std::min(c.wq_lo, c.wq_hi);
    }
  }
  c.BL = (uint32_t)r.getu("-gpgpu_dram_burst_length");
  c.busW = (uint32_t)r.getu("-gpgpu_dram_buswidth");
  c.data_cmd_ratio = std::max<uint32_t>(1, (uint32_t)r.getu("-dram_data_command_freq_ratio"));
  c.dual_bus = (uint32_t)r.getu("-dram_dual_bus_interface");
  c.perfect_mem = r.getb("-gpgpu_perfect_mem") ? 1u : 0u;
  c.simple_dram = r.getb("-gpgpu_simple_dram_model") ? 1u : 0u;
  c.event_skip = r.getb("-sim_event_skip") ? 1u : 0u;
  c.trace_window = (uint32_t)std::max<long long>(0, r.geti("-gpu_trace_window"));
  {
    // CDNA4 memory hierarchy
    c.l1_wr_req_bytes = (uint32_t)r.getu("-sim_l1_write_request_bytes");
    c.single_valu = r.getb("-sim_single_valu") ? 1u : 0u;
    if (c.l1_wr_req_bytes != 64 && c.l1_wr_req_bytes != 128)
      throw OptionError("-sim_l1_write_request_bytes must be 64 or 128");
    c.n_xcd = (uint32_t)r.getu("-sim_xcd");
    c.log2_spx = 0;
    if (c.n_xcd > 1) {
      if (c.n_subpart % c.n_xcd) throw OptionError("-sim_xcd must divide the number of L2 sub-partitions");
      if (c.n_xcd > (uint32_t)kMaxXcd || c.n_xcd > c.n_sm)
        throw OptionError("-sim_xcd: at most " + std::to_string(kMaxXcd) + " XCDs and no more than the SMs");
      const uint32_t spx = c.n_subpart / c.n_xcd;
      if (spx & (spx - 1)) throw OptionError("-sim_xcd: sub-partitions per XCD must be a power of two");
      while ((1u << c.log2_spx) < spx) ++c.log2_spx;
    } else {
      c.n_xcd = 0;
    }
    c.mall_sets = c.mall_assoc = 0;
    const std::string m = strip_ws(r.gets("-sim_mall"));
    if (!m.empty() && m != "none" && m != "0") {
      auto v = split(m, ':');
      if (v.size() != 2) throw OptionError("-sim_mall expects <sets>:<assoc>");
      c.mall_sets = parse_u(v[0], "-sim_mall");
      c.mall_assoc = parse_u(v[1], "-sim_mall");
      if (!c.mall_sets || (c.mall_sets & (c.mall_sets - 1)) || !c.mall_assoc || c.mall_assoc > 64)
        throw OptionError("-sim_mall: sets must be a power of two and 1 <= assoc <= 64");
    }
    c.mall_miss_fs = (uint64_t)r.getu("-sim_mall_miss_latency");  // cycles; fs once the clocks are known
  }
  c.cpu_threads = r.getu("-sim_cpu_threads");
  c.trace_mask = 0;
  if (r.getb("-trace_enabled")) {
    static const std::pair<const char*, uint32_t> streams[] = {
        {"WARP_SCHEDULER", TS_WARP_SCHEDULER},
        {"SCOREBOARD", TS_SCOREBOARD},
        {"MEMORY_PARTITION_UNIT", TS_MEMORY_PARTITION_UNIT},
        {"MEMORY_SUBPARTITION_UNIT", TS_MEMORY_SUBPARTITION_UNIT},
        {"INTERCONNECT", TS_INTERCONNECT},
        {"LIVENESS", TS_LIVENESS}};
    for (auto& tok : split(strip_ws(r.gets("-trace_components")), ',')) {
      if (tok.empty() || tok == "none") continue;
      bool found = false;
      for (auto& s : streams)
        if (tok == s.first || tok == "all") {
          c.trace_mask |= s.second;
          found = true;
        }
      if (!found) throw OptionError("-trace_components: unknown stream " + tok);
    }
  }
  c.trace_sm = (int32_t)r.geti("-trace_sampling_core");
  c.trace_mem = (int32_t)r.geti("-trace_sampling_memory_partition");
  c.trace_cap = 1u << 16;
  c.trace_ev = nullptr;
  c.trace_cnt = nullptr;
  c.bk_index_policy = (uint32_t)r.getu("-dram_bnk_indexing_policy");
  c.bkgrp_index_policy = (uint32_t)r.getu("-dram_bnkgrp_indexing_policy");
  c.atom_size = c.BL * c.busW * (uint32_t)r.getu("-gpgpu_n_mem_per_ctrlr");
  // address decode
  setup_addrdec(c, trim(r.gets("-gpgpu_mem_addr_mapping")), (int)r.geti("-gpgpu_mem_address_mask"));
  {
    uint32_t pi = (uint32_t)r.getu(user_set("-memory_partition_indexing") ? "-memory_partition_indexing"
                                                                           : "-gpgpu_memory_partition_indexing");
    if (pi > 5) throw OptionError("-gpgpu_memory_partition_indexing out of range");
    c.part_index = (uint8_t)pi;
  }
  // clocks
  {
    auto v = split(strip_ws(r.gets("-gpgpu_clock_domains")), ':');
    if (v.size() != 4) throw OptionError("-gpgpu_clock_domains expects 4 frequencies");
    double f[4];
    for (int i = 0; i < 4; ++i) {
      f[i] = atof(v[i].c_str());
      if (f[i] <= 0) throw OptionError("clock frequency must be positive");
    }
    // femtoseconds per cycle
    c.per_core = (uint64_t)llround(1e9 / f[0]);
    c.per_icnt = (uint64_t)llround(1e9 / f[1]);
    c.per_l2 = (uint64_t)llround(1e9 / f[2]);
    c.per_dram = (uint64_t)llround(1e9 / f[3]);
    cfg_set_divs(c);
  }
  c.mall_miss_fs *= c.per_core;
  c.per_core_max = c.per_core;
  if (r.getb("-dvfs_enabled")) {
    const double mr = r.getd("-dvfs_min_clock_ratio");
    if (!(mr > 0.05 && mr <= 1.0)) throw OptionError("-dvfs_min_clock_ratio must be in (0.05, 1]");
    c.per_core_max = (uint64_t)std::ceil((double)c.per_core / mr);
  }
  c.kernel_launch_latency = (uint32_t)std::max<long long>(0, r.geti("-gpgpu_kernel_launch_latency"));
  {
    const long long q = r.geti("-gpgpu_kernel_launch_latency_queued");
    c.kernel_launch_latency_queued = q < 0 ? c.kernel_launch_latency : (uint32_t)q;
  }
  c.tb_launch_latency = (uint32_t)std::max<long long>(0, r.geti("-gpgpu_TB_launch_latency"));
  c.deadlock_window = r.getb("-gpgpu_deadlock_detect") ? 50000 : 0;
  c.max_insn = (uint64_t)std::max<long long>(0, r.geti("-gpgpu_max_insn"));
  c.max_completed_cta = (uint32_t)std::max<long long>(0, r.geti("-gpgpu_max_completed_cta"));
  // interconnect model
  c.icnt_mode = 2;
  if (r.geti("-network_mode") == 1) {
    apply_intersim_config(c, resolve_cfg_path(r, r.gets("-inter_config_file")));
    const uint64_t lc = r.getu("-icnt_link_contention");
    if (lc > 2) throw OptionError("-icnt_link_contention must be 0, 1 (link reservations) or 2 (router model)");
    c.link_contention = (uint16_t)lc;
    if (lc == 2 && c.rt_alloc == 0xff)
      throw OptionError("-icnt_link_contention 2: the .icnt file's sw_allocator is not modelled "
                        "(islip, separable_input_first, separable_output_first, wavefront, rr_wavefront, max_size, pim, loa)");
    // configurations whose channel dependences can form a cycle: the pass
    // would report a routing deadlock (the dateline classes of a torus and
    // the escape / second-leg classes of min_adapt / valiant need two VCs)
    if (lc == 2 && c.rt_vcs < 2 && c.topo == TOPO_TORUS)
      throw OptionError("-icnt_link_contention 2: a torus needs num_vcs >= 2 (dateline classes)");
    if (lc == 2 && c.rt_vcs < 2 && c.rt_route != 0)
      throw OptionError("-icnt_link_contention 2: min_adapt / valiant routing needs num_vcs >= 2");
  } else if (r.geti("-network_mode") != 2) {
    throw OptionError("-network_mode must be 1 (intersim topology) or 2 (local crossbar)");
  }
  cfg_set_divs(c);  // the epoch length is final here
  return c;
}

Occupancy compute_occupancy(const SimCfg& c, const KernelShape& k) {
  Occupancy o{};
  const uint32_t ws = c.warp_size;
  const uint32_t padded = (k.threads_per_cta + ws - 1) / ws * ws;
  const uint32_t wpc = padded / ws;
  uint32_t lim = c.max_cta_per_sm;
  o.limiter = "cta";
  auto take = [&](uint32_t v, const char* why) {
    if (v < lim) {
      lim = v;
      o.limiter = why;
    }
  };
  take(padded ? c.max_threads_per_sm / padded : lim, "threads");
  take(wpc ? (uint32_t)kMaxWarps / wpc : lim, "warps");
  if (k.regs_per_thread) {
    uint32_t per = padded * ((k.regs_per_thread + 3) & ~3u);
    take(per ? c.regs_per_sm / per : lim, "registers");
  }
  uint32_t shmem_cap = c.shmem_per_sm;
  uint32_t l1_kb = 0;
  if (c.adaptive_l1 && c.unified_l1_kb && c.n_shmem_opts) {
    // choose the smallest carve-out that holds the CTAs the other limits allow
    uint32_t want = k.shmem_per_cta * lim;
    uint32_t chosen = c.shmem_opts_kb[c.n_shmem_opts - 1];
    for (uint32_t i = 0; i < c.n_shmem_opts; ++i)
      if (want <= c.shmem_opts_kb[i] * 1024u) {
        chosen = c.shmem_opts_kb[i];
        break;
      }
    shmem_cap = chosen * 1024u;
    o.shmem_kb = chosen;
    l1_kb = c.unified_l1_kb > chosen ? c.unified_l1_kb - chosen : 0;
  }
  if (k.shmem_per_cta) take(shmem_cap / k.shmem_per_cta, "shared memory");
  if (lim == 0) lim = 1;  // reference asserts; a kernel always gets one CTA slot
  o.cta_per_sm = lim;
  o.l1_sets = c.l1.nsets;
  o.l1_assoc = c.l1.assoc;
  if (l1_kb && !c.l1.disabled) {
    uint32_t lines = l1_kb * 1024u / c.l1.line;
    if (lines > (uint32_t)kMaxL1Lines) lines = kMaxL1Lines;
    uint32_t a = lines / c.l1.nsets;
    if (a >= 1) o.l1_assoc = a;
  }
  return o;
}

DriverOpts derive_driver_opts(const OptionRegistry& r) {
  DriverOpts d;
  d.trace_file = r.gets("-trace");
  d.max_cycle = r.geti("-gpgpu_max_cycle");
  d.max_insn = r.geti("-gpgpu_max_insn");
  d.max_cta = (int32_t)r.geti("-gpgpu_max_cta");
  d.max_completed_cta = (int32_t)r.geti("-gpgpu_max_completed_cta");
  d.flush_l1 = r.getb("-gpgpu_flush_l1_cache");
  d.sqc_invalidate = r.getb("-sim_sqc_invalidate_at_launch");
  d.flush_l2 = r.getb("-gpgpu_flush_l2_cache");
  d.l2_kernel_release = r.getb("-sim_l2_kernel_release");
  d.coll_mem_traffic = r.getb("-collective_mem_traffic");
  d.host_launch_interval = r.getu("-sim_host_launch_interval");
  d.first_kernel_latency = r.getu("-sim_first_kernel_latency");
  d.copy_latency_every = r.getb("-sim_copy_latency_every_kernel");
  d.kernel_min_cycles_queued = r.getu("-sim_kernel_min_cycles_queued");
  d.dvfs = r.getb("-dvfs_enabled");
  d.dvfs_min_clock_ratio = r.getd("-dvfs_min_clock_ratio");
  d.deadlock_detect = r.getb("-gpgpu_deadlock_detect");
  d.nccl_allreduce_latency = (int32_t)r.geti("-nccl_allreduce_latency");
  d.collective_model = r.gets("-collective_model");
  d.xgmi_link_gbps = r.getd("-xgmi_link_bandwidth_gbps");
  d.xgmi_latency_ns = r.getd("-xgmi_link_latency_ns");
  d.xgmi_links = (uint32_t)r.getu("-xgmi_links_per_gpu");
  d.coll_slice_bytes = (uint32_t)r.getu("-collective_slice_bytes");
  d.coll_max_channels = (uint32_t)r.getu("-collective_max_channels");
  d.coll_reduce_gbps = r.getd("-collective_reduce_gbps");
  d.concurrent_kernel_sm = r.getb("-gpgpu_concurrent_kernel_sm") ? 1 : 0;
  d.max_concurrent_kernel = (int32_t)r.geti("-gpgpu_max_concurrent_kernel");
  d.trace_prefetch = r.getb("-trace_prefetch");
  d.host_budget_mb = r.getd("-trace_host_budget_mb");
  d.power_in_loop = r.getb("-power_in_loop");
  d.gpu_ingest = r.getb("-gpu_ingest");
  d.gpu_ingest_min = (uint64_t)r.getu("-gpu_ingest_min_insts");
  d.power_enabled = r.getb("-power_simulation_enabled");
  d.power_xml = r.gets("-accelwattch_xml_file");
  {
    // legacy GPUWattch configs (SM2_GTX480) name their XML with -gpuwattch_xml_file
    const OptionRegistry::Opt* aw = r.find("-accelwattch_xml_file");
    const OptionRegistry::Opt* gw = r.find("-gpuwattch_xml_file");
    if (gw && gw->parsed && !(aw && aw->parsed)) d.power_xml = r.gets("-gpuwattch_xml_file");
    d.power_xml = resolve_cfg_path(r, d.power_xml);
  }
  d.power_mode = (int32_t)r.geti("-power_simulation_mode");
  d.hw_perf_file = r.gets("-hw_perf_file_name");
  d.hw_perf_bench = r.gets("-hw_perf_bench_name");
  {
    static const char* hw[17] = {"L1_RH", "L1_RM", "L1_WH", "L1_WM", "CC_ACC", "SHARED_ACC", "DRAM_RD", "DRAM_WR",
                                 "L2_RH", "L2_RM", "L2_WH", "L2_WM", "NOC", "PIPE_DUTY", "NUM_SM_IDLE", "CYCLES",
                                 "VOLTAGE"};
    for (int i = 0; i < 17; ++i) d.hybrid_use_sim[i] = r.getb(std::string("-accelwattch_hybrid_perfsim_") + hw[i]);
  }
  d.power_trace = r.getb("-power_trace_enabled");
  d.steady_power = r.getb("-steady_power_levels_enabled");
  {
    auto v = split(strip_ws(r.gets("-steady_state_definition")), ':');
    if (v.size() == 2) {
      d.steady_dev_pct = atof(v[0].c_str());
      d.steady_samples = (uint32_t)std::max(1, atoi(v[1].c_str()));
    }
  }
  d.power_report_file = r.gets("-power_report_file");
  d.memlatency_stat = (int32_t)r.geti("-gpgpu_memlatency_stat");
  d.visualizer = r.getb("-visualizer_enabled");
  d.visualizer_file = r.gets("-visualizer_outputfile");
  if (d.visualizer_file.empty()) d.visualizer_file = "gpgpusim_visualizer.log";
  d.checkpoint_option = (int32_t)r.geti("-checkpoint_option");
  d.checkpoint_kernel = (int32_t)r.geti("-checkpoint_kernel");
  d.resume_option = (int32_t)r.geti("-resume_option");
  d.resume_kernel = (int32_t)r.geti("-resume_kernel");
  d.checkpoint_dir = r.gets("-checkpoint_path");
  {
    auto v = split(strip_ws(r.gets("-gpgpu_runtime_stat")), ':');
    d.stat_sample_freq = v.empty() || v[0].empty() ? 500 : parse_u(v[0], "-gpgpu_runtime_stat");
  }
  d.engine = r.gets("-sim_engine");
  d.check_interval = r.getu("-sim_check_interval");
  d.check_primary = r.gets("-sim_check_primary");
  d.check_corrupt_at = r.getu("-sim_check_corrupt_at");
  d.check_corrupt_mailbox = r.getu("-sim_check_corrupt_mailbox");
  d.trace_enabled = r.getb("-trace_enabled");
  d.trace_components = r.gets("-trace_components");
  d.trace_sampling_core = (int32_t)r.geti("-trace_sampling_core");
  d.sim_epochs_per_launch = (uint32_t)r.getu("-sim_epochs_per_launch");
  {
    const char* env = getenv("GPGPUSIM_DEBUG");
    d.debug = r.getb("-sim_debug") || (env && *env && *env != '0') || r.getu("-sim_break_cycle") > 0;
  }
  d.debug_script = r.gets("-sim_debug_script");
  d.debug_step = r.getu("-sim_debug_step");
  d.break_cycle = r.getu("-sim_break_cycle");
  return d;
}

}  // namespace asim
