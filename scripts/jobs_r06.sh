#!/bin/bash
# Round-6 GPU evidence jobs (run through gpurun): bash scripts/jobs_r06.sh <name>.
# Each job is a list of scripts/gpu_job.sh steps; logs land in gpurun_out/, the
# summaries judged are copied into profiles/ (named after the job).
set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"                 # headline, K = 50
H="--configs none --no-cpu-baseline --no-conv"                            # headline, K = 20 (driver shape)
M="--only C3x1M --no-cpu-baseline --no-conv --steps 20 --warmup 1 --ar-probe 0"   # over-cache 1M
A="--no-cpu-baseline --no-conv --steps 10 --warmup 1"                     # one secondary config
S8="--only C3s8 --no-cpu-baseline --no-conv --steps 20"                   # the 8-GPU per-rank slice
SQ="SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU_FLOPS_FP64,SQ_INSTS_SALU"
NOPARK="PHX_LANE_DEFS=PHX_FZR2_NO_PARK"
J="bash scripts/gpu_job.sh"
case "$1" in
  s8)  # the two-wave fused build with its round data parked in LDS (no spill): parity, then A/B against the
       # round-5 build (same box, alternating), kernel trace, PMC bytes
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_bench_settings.py" && \
       $J "bench:r06_s8_h1:$H --ar-probe 0" && env $NOPARK $J "bench:r06_s8_h1_nopark:$H --ar-probe 0" && \
       $J "bench:r06_s8_h2:$H --ar-probe 0" && env $NOPARK $J "bench:r06_s8_h2_nopark:$H --ar-probe 0" && \
       $J "bench:r06_s8_1m:$M" && env $NOPARK $J "bench:r06_s8_1m_nopark:$M" && \
       $J "prof:r06_s8_prof:$H --ar-probe 0" "pmc:r06_pmc_c3_fetch:FETCH_SIZE:$B" "pmc:r06_pmc_c3_write:WRITE_SIZE:$B" ;;
  s9)  # C4: Compute_Xbar + Update_W + convergence_diff of small batches in one block (k_small_xw): the whole
       # suite, then C4 A/B against the two-kernel path (PHX_SMALL_XW=0), kernel trace
       $J "test:tests" && \
       $J "bench:r06_s9_c4:--only C4 $A" && PHX_SMALL_XW=0 $J "bench:r06_s9_c4_old:--only C4 $A" && \
       $J "bench:r06_s9_c4b:--only C4 $A" && PHX_SMALL_XW=0 $J "bench:r06_s9_c4b_old:--only C4 $A" && \
       $J "prof:r06_s9_c4_prof:--only C4 $A" ;;
  s10) # k_small_xw with its run sums in LDS; C4 with the kernel timing in a run of its own (the default configs path)
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_distributed_gpu.py tests/test_hydro.py" && \
       $J "bench:r06_s10_c4:--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1" && \
       PHX_SMALL_XW=0 $J "bench:r06_s10_c4_old:--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1" && \
       $J "bench:r06_s10_c4b:--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1" && \
       $J "prof:r06_s10_c4_prof:--only C4 $A" ;;
  s11) # sparse configs: the split level 2 layout (four workgroups per CU) against the default, C5a / C5b; C5b's
       # setup trace (the lazy PDHG step size: no k_norm)
       Q="--configs C5a,C5b --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "bench:r06_s11_sp:$Q" && PHX_SP_SPLIT=2 $J "bench:r06_s11_sp_split2:$Q" && \
       $J "prof:r06_s11_c5b_prof:--only C5b $A" ;;
  s12) # the per-iteration glue kernels by element / slot chunk (k_begin_vec, k_ph_terms2, k_update_w_seg2, k_xbar's
       # fold by slot), split level 2 for the sparse-primary problems: parity, C5a / C5b / C2, C5b trace
       Q="--configs C2,C5a,C5b --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests/test_netdes.py tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" && \
       $J "bench:r06_s12_sp:$Q" "prof:r06_s12_c5b_prof:--only C5b $A" ;;
  s13) # C5a / C2 kernel traces (where their steps go after the glue-kernel changes)
       $J "prof:r06_s13_c5a_prof:--only C5a $A" "prof:r06_s13_c2_prof:--only C2 $A" ;;
  s14) # the glue kernels by slot chunk from 16 slots (C2), the counters zeroed by the PH-terms kernel
       Q="--configs C2,C5a,C5b --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests/test_netdes.py tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" && \
       $J "bench:r06_s14_sp:$Q" "prof:r06_s14_c2_prof:--only C2 $A" ;;
  s15) # the whole GPU suite, then the driver's default command
       $J "test:tests" && $J "bench:r06_s15_default:--detail gpurun_out/r06_s15_default_detail.json" ;;
  s16) # the per-rank slice (C3s8) and the headline: kernel traces of the timed windows
       $J "prof:r06_s16_c3s8_prof:$S8" "prof:r06_s16_prof:$H --ar-probe 0" ;;
  s17) # the interior point's per-iteration arrays parked in LDS, the predictor's terms without the zero
       # shift / second-order terms, the KKT check from iteration 6: parity, then Iter0 A/B (PHX_IPM_NO_PARK)
       IPMNP="PHX_LANE_DEFS=PHX_IPM_NO_PARK"
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py" && \
       $J "run:r06_s17_rcp_acc:scripts/micro/rcp_acc" && \
       $J "bench:r06_s17_h1:$H --ar-probe 0" && env $IPMNP $J "bench:r06_s17_h1_np:$H --ar-probe 0" && \
       $J "bench:r06_s17_h2:$H --ar-probe 0" && env $IPMNP $J "bench:r06_s17_h2_np:$H --ar-probe 0" && \
       $J "bench:r06_s17_1m:$M" && env $IPMNP $J "bench:r06_s17_1m_np:$M" && \
       $J "bench:r06_s17_c4:--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1" && \
       env $IPMNP $J "bench:r06_s17_c4_np:--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1" && \
       $J "prof:r06_s17_prof:$H --ar-probe 0" ;;
  s18) # the first PH iteration as a fused launch with the rescue round budget (PHX_FUSED_FIRST=1) against the
       # unfused body (k_xbar + k_update_w_seg + warm pass + rescue list + gated cold pass): A/B, traces
       FF="PHX_FUSED_FIRST=1"
       $J "bench:r06_s18_h1:$H --ar-probe 0" && env $FF $J "bench:r06_s18_h1_ff:$H --ar-probe 0" && \
       $J "bench:r06_s18_h2:$H --ar-probe 0" && env $FF $J "bench:r06_s18_h2_ff:$H --ar-probe 0" && \
       $J "bench:r06_s18_1m:$M" && env $FF $J "bench:r06_s18_1m_ff:$M" && \
       $J "bench:r06_s18_s8:--configs C3s8 --no-cpu-baseline --no-conv --ar-probe 0" && \
       env $FF $J "bench:r06_s18_s8_ff:--configs C3s8 --no-cpu-baseline --no-conv --ar-probe 0" && \
       env $FF $J "prof:r06_s18_prof_ff:$H --ar-probe 0" ;;
  s19) # batches of at most one lane block per CU: the interior point parks all its per-iteration arrays (96 KB
       # budget): parity, C4 / C3s8 A/B against the 40 KB budget
       P40="PHX_LANE_DEFS=PHX_IPM_PARK_BYTES=40960"
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py tests/test_distributed_gpu.py" && \
       $J "bench:r06_s19_a1:$Q" && env $P40 $J "bench:r06_s19_a1_40:$Q" && \
       $J "bench:r06_s19_a2:$Q" && env $P40 $J "bench:r06_s19_a2_40:$Q" && \
       $J "prof:r06_s19_c4_prof:--only C4 $A" "prof:r06_s19_c3s8_prof:$S8" ;;
  s20) # C4: bounded multi-change rescue updates (PHX_MULTI_THETA, a JIT define) on the GPU, A/B against the
       # single-change rounds, alternating on one box
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       T2="PHX_LANE_DEFS=PHX_MULTI_THETA=0.2 PHX_MULTI_ROUNDS=4"
       T5="PHX_LANE_DEFS=PHX_MULTI_THETA=0.5 PHX_MULTI_ROUNDS=4"
       T8="PHX_LANE_DEFS=PHX_MULTI_THETA=0.2 PHX_MULTI_ROUNDS=8"
       $J "bench:r06_s20_a:$Q" && env "$T2" $J "bench:r06_s20_t2:$Q" && env "$T5" $J "bench:r06_s20_t5:$Q" && \
       env "$T8" $J "bench:r06_s20_t8:$Q" && $J "bench:r06_s20_b:$Q" && env "$T2" $J "bench:r06_s20_t2b:$Q" ;;
  s21) # where the sparse solver's time goes: phase clocks (PHX_SP_PROF) of C5a's leftover pass and C5b
       PHX_SP_PROF=1 $J "bench:r06_s21_c5a_spprof:--only C5a $A" && PHX_SP_PROF=1 $J "bench:r06_s21_c5b_spprof:--only C5b $A" ;;
  s22) # bounded multi-change updates: the theta / rounds neighbourhood on C4, and their effect on farmer (the
       # headline, C3s8, C1: the rescue pass of the first PH iteration); the sparse phase clocks; a C3s8 trace
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       F="--configs C3s8,C1 --no-cpu-baseline --no-conv --ar-probe 0"
       D="PHX_LANE_DEFS=PHX_MULTI_THETA=0.2 PHX_MULTI_ROUNDS=4"
       env "PHX_LANE_DEFS=PHX_MULTI_THETA=0.1 PHX_MULTI_ROUNDS=4" $J "bench:r06_s22_t1r4:$Q" && \
       env "PHX_LANE_DEFS=PHX_MULTI_THETA=0.3 PHX_MULTI_ROUNDS=4" $J "bench:r06_s22_t3r4:$Q" && \
       env "PHX_LANE_DEFS=PHX_MULTI_THETA=0.2 PHX_MULTI_ROUNDS=2" $J "bench:r06_s22_t2r2:$Q" && \
       env "PHX_LANE_DEFS=PHX_MULTI_THETA=0.2 PHX_MULTI_ROUNDS=6" $J "bench:r06_s22_t2r6:$Q" && \
       env "PHX_LANE_DEFS=PHX_MULTI_THETA=0.2 PHX_MULTI_ROUNDS=3" $J "bench:r06_s22_t2r3:$Q" && \
       $J "bench:r06_s22_f:$F" && env "$D" $J "bench:r06_s22_f_t2:$F" && \
       $J "bench:r06_s22_f2:$F" && env "$D" $J "bench:r06_s22_f2_t2:$F" && \
       PHX_SP_PROF=1 $J "bench:r06_s22_c5a_spprof:--only C5a $A" && PHX_SP_PROF=1 $J "bench:r06_s22_c5b_spprof:--only C5b $A" && \
       $J "prof:r06_s22_c3s8_prof:$S8" ;;
  s23) # the multi-change setting as C4's solver option (lane_multi_theta, compiled with the problem): parity
       # tests, then the default configs path for C4 twice
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests/test_engine_emu.py tests/test_bench_settings.py tests/test_gpu_parity.py::test_aircond_bf10x10x10_gpu" && \
       $J "bench:r06_s23_c4:$Q" && $J "bench:r06_s23_c4b:$Q" ;;
  s26) # the bench's collector handling (a full collection + freeze before each warm-up, the collector off in
       # the timed regions) against the collector left on (PHX_BENCH_GC=1), alternating on one box
       H2="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0"
       $J "bench:r06_s26_a1:$H2" && PHX_BENCH_GC=1 $J "bench:r06_s26_g1:$H2" && \
       $J "bench:r06_s26_a2:$H2" && PHX_BENCH_GC=1 $J "bench:r06_s26_g2:$H2" && \
       $J "bench:r06_s26_a3:$H2" && PHX_BENCH_GC=1 $J "bench:r06_s26_g3:$H2" ;;
  s27) # host time inside the timed region after the collector change (host_marks), C4's kernel trace with the
       # multi-change setting, the headline's kernel + HIP runtime trace
       $J "py:r06_s27_marks:scripts/host_marks.py 100000 20 5" "prof:r06_s27_c4_prof:--only C4 $A" \
          "trace:r06_s27_trace:$H --ar-probe 0" ;;
  s29) # the headline's kernel-timing events in a second timed run (the metric's run records none) against
       # the round-5 form (--kernel-timing-inline), alternating on one box
       $J "bench:r06_s29_a1:$H --ar-probe 0" && $J "bench:r06_s29_i1:$H --ar-probe 0 --kernel-timing-inline" && \
       $J "bench:r06_s29_a2:$H --ar-probe 0" && $J "bench:r06_s29_i2:$H --ar-probe 0 --kernel-timing-inline" && \
       $J "bench:r06_s29_a3:$H --ar-probe 0" && $J "bench:r06_s29_i3:$H --ar-probe 0 --kernel-timing-inline" && \
       $J "bench:r06_s29_m:$M" ;;
  s30) # the rescue list and its cold pass in one launch (phx_lane_list_all) against the three launches
       # (PHX_LIST_ALL=0): parity, then the headline and 1M alternating on one box, and a kernel trace
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py tests/test_distributed_gpu.py tests/test_engine_emu.py" && \
       $J "bench:r06_s30_a1:$H --ar-probe 0" && PHX_LIST_ALL=0 $J "bench:r06_s30_o1:$H --ar-probe 0" && \
       $J "bench:r06_s30_a2:$H --ar-probe 0" && PHX_LIST_ALL=0 $J "bench:r06_s30_o2:$H --ar-probe 0" && \
       $J "bench:r06_s30_a3:$H --ar-probe 0" && PHX_LIST_ALL=0 $J "bench:r06_s30_o3:$H --ar-probe 0" && \
       $J "bench:r06_s30_m:$M" && PHX_LIST_ALL=0 $J "bench:r06_s30_mo:$M" && \
       $J "prof:r06_s30_prof:$H --ar-probe 0" ;;
  s31) # k_small_xw with every load at entry (slot columns by value, the node table and the ranks' counts
       # prefetched before the gate): parity, C4 twice, C4 kernel trace
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py tests/test_engine_emu.py tests/test_bench_settings.py" && \
       $J "bench:r06_s31_c4:$Q" && $J "bench:r06_s31_c4b:$Q" && $J "prof:r06_s31_c4_prof:--only C4 $A" ;;
  s33) # the hybrid first iteration with its first pass fused (k_xbar + one fused launch + the rescue list +
       # the decision kernel) against the unfused body (PHX_HYBRID_FUSED=0): the whole suite, then A/B
       # alternating on one box (headline, C3s8, 1M)
       HF="PHX_HYBRID_FUSED=0"
       $J "test:tests" && \
       $J "bench:r06_s33_a1:$H --ar-probe 0" && env $HF $J "bench:r06_s33_o1:$H --ar-probe 0" && \
       $J "bench:r06_s33_a2:$H --ar-probe 0" && env $HF $J "bench:r06_s33_o2:$H --ar-probe 0" && \
       $J "bench:r06_s33_a3:$H --ar-probe 0" && env $HF $J "bench:r06_s33_o3:$H --ar-probe 0" && \
       $J "bench:r06_s33_s8:--configs C3s8 --no-cpu-baseline --no-conv --ar-probe 0" && \
       env $HF $J "bench:r06_s33_s8o:--configs C3s8 --no-cpu-baseline --no-conv --ar-probe 0" && \
       $J "bench:r06_s33_m:$M" && env $HF $J "bench:r06_s33_mo:$M" && \
       $J "prof:r06_s33_prof:$H --ar-probe 0" ;;
  s34) # C4's lane-solver round budgets with the multi-change setting: as_rounds / rescue_rounds sweep
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "bench:r06_s34_d:$Q" && \
       $J "bench:r06_s34_a3:$Q --so {\"as_rounds\":3}" && $J "bench:r06_s34_a6:$Q --so {\"as_rounds\":6}" && \
       $J "bench:r06_s34_a8:$Q --so {\"as_rounds\":8}" && $J "bench:r06_s34_r16:$Q --so {\"rescue_rounds\":16}" && \
       $J "bench:r06_s34_r64:$Q --so {\"rescue_rounds\":64}" && $J "bench:r06_s34_d2:$Q" ;;
  s37) # C4: the warm passes' full-update rounds (single_after 3 by default) with the multi-change setting
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "bench:r06_s37_d:$Q" && PHX_WARM_SINGLE_AFTER=1 $J "bench:r06_s37_w1:$Q" && \
       PHX_WARM_SINGLE_AFTER=2 $J "bench:r06_s37_w2:$Q" && PHX_WARM_SINGLE_AFTER=4 $J "bench:r06_s37_w4:$Q" && \
       $J "bench:r06_s37_d2:$Q" && PHX_WARM_SINGLE_AFTER=2 $J "bench:r06_s37_w2b:$Q" ;;
  s38) # C4 / C3s8: phx_lane_all re-loading its data per round (PHX_ALL_RELOAD, a JIT define: fewer registers,
       # aircond's 740 B/lane spill) against the register build, alternating
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       R="PHX_LANE_DEFS=PHX_ALL_RELOAD"
       $J "bench:r06_s38_a:$Q" && env $R $J "bench:r06_s38_r:$Q" && \
       $J "bench:r06_s38_a2:$Q" && env $R $J "bench:r06_s38_r2:$Q" ;;
  s39) # phx_lane_all's re-loading build where the register build spills (aircond) + k_small_xw's scans
       # without key shuffles: parity, C4 / C3s8 twice, C4 kernel trace
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py tests/test_engine_emu.py tests/test_bench_settings.py tests/test_distributed_gpu.py" && \
       $J "bench:r06_s39_a:$Q" && $J "bench:r06_s39_b:$Q" && $J "prof:r06_s39_c4_prof:--only C4 $A" ;;
  s40) # k_small_xw's run scans as DPP steps (no ds_bpermute), prev_left loaded at entry: parity, C4 twice, C4 trace
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py tests/test_engine_emu.py tests/test_bench_settings.py tests/test_distributed_gpu.py" && \
       $J "bench:r06_s40_a:$Q" && $J "bench:r06_s40_b:$Q" && $J "prof:r06_s40_c4_prof:--only C4 $A" ;;
  s41) # + k_small_xw's node fold with one LDS round trip per entry, Iter0's copies and sums in one launch for
       # S <= 8192 (k_iter0_keep1): parity, C4 twice, C4 trace
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests" && \
       $J "bench:r06_s41_a:$Q" && $J "bench:r06_s41_b:$Q" && $J "prof:r06_s41_c4_prof:--only C4 $A" ;;
  s42) # k_small_xw: the node fold four wavefronts per LDS round trip (s41's sixteen raised it to 17.3 us), the
       # convergence sum unrolled in registers (no scratch); C4 twice, C4 trace
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "bench:r06_s42_a:$Q" && $J "bench:r06_s42_b:$Q" && $J "prof:r06_s42_c4_prof:--only C4 $A" ;;
  s43) # phx_lane_all_pk (the warm and rescue rounds' data parked in LDS) against phx_lane_all_rl: the aircond
       # parity tests with the park build forced, C4 alternating, C4 trace of the park build
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       P="PHX_ALL_BUILD=park"
       env $P $J "test:tests -k aircond" && \
       env $P $J "bench:r06_s43_p:$Q" && $J "bench:r06_s43_r:$Q" && env $P $J "bench:r06_s43_p2:$Q" && \
       $J "bench:r06_s43_r2:$Q" && env $P $J "prof:r06_s43_c4_prof:--only C4 $A" ;;
  s44) # phx_lane_all_pk the default where phx_lane_all spills; the unfused loop's tail copies as one kernel
       # (k_tail_copy): the whole GPU suite, C4 / C3s8 twice, C4 trace
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests" && $J "bench:r06_s44_a:$Q" && $J "bench:r06_s44_b:$Q" && $J "prof:r06_s44_c4_prof:--only C4 $A" ;;
  s45) # s44 rebuilt (s44's library predates the park default): the aircond and iterk tests, C4 / C3s8 twice, C4 trace
       Q="--configs C4,C3s8 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "test:tests -k aircond" && $J "bench:r06_s45_a:$Q" && $J "bench:r06_s45_b:$Q" && \
       $J "prof:r06_s45_c4_prof:--only C4 $A" ;;
  s47) # C4 on the final sources, three runs on one box (the box-to-box spread of the step)
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "bench:r06_s47_a:$Q" && $J "bench:r06_s47_b:$Q" && $J "bench:r06_s47_c:$Q" ;;
  s48) # C4 inside the default run against C4 alone, one box (is the default run's C4 slower by its order?)
       Q="--configs C4 --no-cpu-baseline --no-conv --ar-probe 0 --steps 10 --warmup 1"
       $J "bench:r06_s48_def:" && $J "bench:r06_s48_c4:$Q" && $J "bench:r06_s48_c4b:$Q" ;;
  final) # the round's evidence: the whole GPU suite, smoke, the driver's default command, kernel traces
       $J "test:tests" && $J "py:r06_final_smoke:scripts/run_smoke.py" "bench:r06_final_default:--detail gpurun_out/r06_final_default_detail.json" \
          "prof:r06_final_prof:$H --ar-probe 0" "prof:r06_final_c3s8_prof:$S8" "prof:r06_final_1m_prof:$M" \
          "prof:r06_final_c2_prof:--only C2 $A" "prof:r06_final_c4_prof:--only C4 $A" "prof:r06_final_c5a_prof:--only C5a $A" \
          "prof:r06_final_c5b_prof:--only C5b $A" ;;
  pmc1) # PMC passes on the final kernels (one counter group per pass): the lane kernels
       $J "pmc:r06_pmc_c3_fetch:FETCH_SIZE:$B" "pmc:r06_pmc_c3_write:WRITE_SIZE:$B" "pmc:r06_pmc_c3_sq:$SQ:$B" \
          "pmc:r06_pmc_s8_fetch:FETCH_SIZE:$S8" "pmc:r06_pmc_s8_write:WRITE_SIZE:$S8" "pmc:r06_pmc_s8_sq:$SQ:$S8" \
          "pmc:r06_pmc_1m_fetch:FETCH_SIZE:$M" "pmc:r06_pmc_1m_write:WRITE_SIZE:$M" \
          "pmc:r06_pmc_c4_fetch:FETCH_SIZE:--only C4 $A" "pmc:r06_pmc_c4_write:WRITE_SIZE:--only C4 $A" ;;
  pmc2) # ... the workgroup and sparse solvers
       $J "pmc:r06_pmc_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r06_pmc_c2_write:WRITE_SIZE:--only C2 $A" \
          "pmc:r06_pmc_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r06_pmc_c5a_write:WRITE_SIZE:--only C5a $A" \
          "pmc:r06_pmc_c5b_fetch:FETCH_SIZE:--only C5b $A" "pmc:r06_pmc_c5b_write:WRITE_SIZE:--only C5b $A" ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
