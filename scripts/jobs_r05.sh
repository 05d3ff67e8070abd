#!/bin/bash
# Round-5 GPU evidence jobs (run through gpurun): bash scripts/jobs_r05.sh <name>.
# Each job is a list of scripts/gpu_job.sh steps; logs land in gpurun_out/, the
# summaries judged are copied into profiles/ (named after the job).
set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"                 # headline, K = 50
H="--configs none --no-cpu-baseline --no-conv"                            # headline, K = 20 (driver shape)
M="--only C3x1M --no-cpu-baseline --no-conv --steps 20 --warmup 1 --ar-probe 0"   # over-cache 1M
A="--no-cpu-baseline --no-conv --steps 10 --warmup 1"                     # one secondary config
S8="--only C3s8 --no-cpu-baseline --no-conv --steps 20"                   # the 8-GPU per-rank slice
SQ="SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU_FLOPS_FP64,SQ_INSTS_SALU"
J="bash scripts/gpu_job.sh"
case "$1" in
  s1)  # the whole GPU suite, then the driver's default command (compact line)
       $J "test:tests" && $J "bench:r05_s1_default:--detail gpurun_out/r05_s1_default_detail.json" ;;
  s2)  # the compacting fused kernel: parity, then headline / per-rank slice / 1M against PHX_FZC=0 (same box)
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_bench_settings.py" "bench:r05_s2_bench:$H" "bench:r05_s2_c3s8:$S8" \
          "bench:r05_s2_1m:$M" && \
       PHX_FZC=0 $J "bench:r05_s2_bench_fz1:$H" "bench:r05_s2_c3s8_fz1:$S8" "bench:r05_s2_1m_fz1:$M" && \
       $J "prof:r05_s2_prof:$H --ar-probe 0" ;;
  s3)  # the workgroup / sparse solvers after the XCD-aware block remap: time, kernel trace, HBM bytes
       $J "bench:r05_s3_c2:--only C2 $A" "bench:r05_s3_c5a:--only C5a $A" "bench:r05_s3_c5b:--only C5b $A" \
          "prof:r05_s3_c2_prof:--only C2 $A" "prof:r05_s3_c5a_prof:--only C5a $A" \
          "pmc:r05_pmc_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r05_pmc_c2_write:WRITE_SIZE:--only C2 $A" \
          "pmc:r05_pmc_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r05_pmc_c5a_write:WRITE_SIZE:--only C5a $A" \
          "pmc:r05_pmc_c5b_fetch:FETCH_SIZE:--only C5b $A" "pmc:r05_pmc_c5b_write:WRITE_SIZE:--only C5b $A" ;;
  s4)  # where a fused wave's time goes: phase stamps by most rounds; the clock under load (GRBM)
       PHX_LANE_STAMPS=1 $J "bench:r05_s4_stamps:$H --ar-probe 0" "bench:r05_s4_c3s8_stamps:$S8" "bench:r05_s4_1m_stamps:$M" && \
       $J "pmc:r05_s4_grbm:GRBM_GUI_ACTIVE,GRBM_COUNT:$H --ar-probe 0" "pmc:r05_s4_c3s8_grbm:GRBM_GUI_ACTIVE,GRBM_COUNT:$S8" ;;
  s5)  # two waves per SIMD with register-resident rounds (PHX_FZR2=1) against the one-wave build, same box
       $J "bench:r05_s5_bench:$H" "bench:r05_s5_1m:$M" && \
       PHX_FZR2=1 $J "bench:r05_s5_bench_r2:$H" "bench:r05_s5_1m_r2:$M" && \
       PHX_FZR2=1 PHX_LANE_STAMPS=1 $J "bench:r05_s5_stamps_r2:$H --ar-probe 0" ;;
  s7)  # the two-wave build by default; post-solve values parked in LDS (JIT define), same box
       $J "test:tests/test_gpu_parity.py -k fused" "bench:r05_s7_bench:$H" "bench:r05_s7_1m:$M" && \
       PHX_LANE_DEFS=PHX_FZ_LDS_KEEP $J "bench:r05_s7_bench_keep:$H" "bench:r05_s7_1m_keep:$M" && \
       $J "bench:r05_s7_bench_b:$H" ;;
  s8)  # the headline's timed region on the GPU timeline (kernel trace + HIP API trace)
       $J "prof:r05_s8_prof:$H --ar-probe 0" "trace:r05_s8_trace:$H --ar-probe 0" ;;
  s9)  # the host's share of the timed region (wall stamps + cProfile)
       $J "py:r05_s9_cprof:scripts/timed_cprof.py" ;;
  s10) # the host's timed-region call tree (every PHBase/SPOpt/SPBase method and ABI call)
       $J "py:r05_s10_wall:scripts/iter0_wall.py" ;;
  s11) # Iter0's interior point at two waves per SIMD (PHX_COLD_WAVES=2, spills) against one, same box
       $J "bench:r05_s11_bench:$H --ar-probe 0" "bench:r05_s11_1m:$M" && \
       PHX_COLD_WAVES=2 $J "bench:r05_s11_bench_cw2:$H --ar-probe 0" "bench:r05_s11_1m_cw2:$M" \
          "prof:r05_s11_prof_cw2:$H --ar-probe 0" ;;
  s12) # the workgroup solver's phase clocks in the device loop (C2, C5a)
       PHX_WG_PROF=1 $J "bench:r05_s12_c2_wgprof:--only C2 $A" "bench:r05_s12_c5a_wgprof:--only C5a $A" ;;
  s13) # the workgroup mode's in-stream sparse step: parity (workgroup / sparse / trajectories), C2 / C5a against the stop (same box)
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_bench_settings.py tests/test_sslp.py" \
          "bench:r05_s13_c2:--only C2 $A" "bench:r05_s13_c5a:--only C5a $A" && \
       PHX_WG_SP_INLINE=0 $J "bench:r05_s13_c2_stop:--only C2 $A" "bench:r05_s13_c5a_stop:--only C5a $A" ;;
  s14) # C4 (aircond 10x10x10): kernel trace of the timed iterations
       $J "prof:r05_s14_c4_prof:--only C4 $A" "bench:r05_s14_c4:--only C4 $A" ;;
  s15) # C2 with one workgroup round in the first PH iteration (wg_first) against eight, same box
       $J "test:tests/test_bench_settings.py tests/test_gpu_parity.py -k workgroup" \
          "bench:r05_s15_c2:--only C2 $A" "bench:r05_s15_c2_wf0:--only C2 $A --so {\"wg_first\":0}" ;;
  s16) # the whole GPU suite, then the driver's default command
       $J "test:tests" && $J "bench:r05_s16_default:--detail gpurun_out/r05_s16_default_detail.json" ;;
  s17) # the workgroup solver's split layout with the shared pattern / A (PHX_WG_SPLIT=1): parity, C5a / C2 against the all-LDS layout, HBM bytes
       PHX_WG_SPLIT=1 $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s17_c5a_split:--only C5a $A" "bench:r05_s17_c2_split:--only C2 $A" \
          "pmc:r05_pmc_c5a_split_fetch:FETCH_SIZE:--only C5a $A" "pmc:r05_pmc_c5a_split_write:WRITE_SIZE:--only C5a $A" && \
       $J "bench:r05_s17_c5a:--only C5a $A" "bench:r05_s17_c2:--only C2 $A" ;;
  s18) # workgroup solver: a quad per row + (P+reg)^-1 per column, the split layout by default on C5a; sparse solver:
       # separator rows / Schur diagonal / msolve links a quad each, readlane substitution -- parity, C5a / C2 / C5b (+ all-LDS C5a)
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s18_c5a:--only C5a $A" "bench:r05_s18_c2:--only C2 $A" "bench:r05_s18_c5b:--only C5b $A" && \
       PHX_WG_SPLIT=0 $J "bench:r05_s18_c5a_lds:--only C5a $A" ;;
  s19) # workgroup solver: the long Schur pairs a quad each; phase clocks (PHX_WG_PROF) of C2 / C5a
       $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_gpu_parity.py" \
          "bench:r05_s19_c2:--only C2 $A" "bench:r05_s19_c5a:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s19_c2_wgprof:--only C2 $A" "bench:r05_s19_c5a_wgprof:--only C5a $A" ;;
  s20) # workgroup solver: refinement sub-phase clocks (C2, C5a); C2 with the blocked MFMA factor (PHX_WG_BLK=1) against the scalar one
       PHX_WG_PROF=1 $J "bench:r05_s20_c2_wgprof:--only C2 $A" "bench:r05_s20_c5a_wgprof:--only C5a $A" && \
       PHX_WG_BLK=1 $J "bench:r05_s20_c2_blk1:--only C2 $A" && PHX_WG_BLK=1 PHX_WG_PROF=1 $J "bench:r05_s20_c2_blk1_wgprof:--only C2 $A" && \
       $J "bench:r05_s20_c2:--only C2 $A" ;;
  s21) # workgroup phase clocks accumulated in LDS (one global add per workgroup): C2 (scalar, blocked) / C5a, and C2 unprofiled
       PHX_WG_PROF=1 $J "bench:r05_s21_c2_wgprof:--only C2 $A" "bench:r05_s21_c5a_wgprof:--only C5a $A" && \
       PHX_WG_BLK=1 PHX_WG_PROF=1 $J "bench:r05_s21_c2_blk1_wgprof:--only C2 $A" && $J "bench:r05_s21_c2:--only C2 $A" ;;
  s22) # (measured and reverted) the refinement by one-wavefront substitution with the factor instead of L^-1: C2 / C5a + phase clocks
       $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py tests/test_wg_blk.py" \
          "bench:r05_s22_c2:--only C2 $A" "bench:r05_s22_c5a:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s22_c2_wgprof:--only C2 $A" "bench:r05_s22_c5a_wgprof:--only C5a $A" ;;
  s23) # workgroup solver: scalar factor + blocked MFMA inverse (BLK 0) -- parity, C2; C5a blocked (default) against BLK 0; phase clocks
       $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py tests/test_wg_blk.py" \
          "bench:r05_s23_c2:--only C2 $A" "bench:r05_s23_c5a:--only C5a $A" && \
       PHX_WG_BLK=0 $J "bench:r05_s23_c5a_blk0:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s23_c2_wgprof:--only C2 $A" && PHX_WG_BLK=0 PHX_WG_PROF=1 $J "bench:r05_s23_c5a_blk0_wgprof:--only C5a $A" ;;
  s24) # sparse solver phase clocks (PHX_SP_PROF): C5b (Iter0 interior point + warm rounds), C5a; C2 workgroup round budget 4 / 6 against 8
       $J "test:tests/test_netdes.py tests/test_sslp.py" && \
       PHX_SP_PROF=1 $J "bench:r05_s24_c5b_spprof:--only C5b $A" "bench:r05_s24_c5a_spprof:--only C5a $A" && \
       $J "bench:r05_s24_c2_w4:--only C2 $A --so {\"wg_warm\":4,\"wg_first\":1}" "bench:r05_s24_c2_w6:--only C2 $A --so {\"wg_warm\":6,\"wg_first\":1}" \
          "bench:r05_s24_c2:--only C2 $A" ;;
  s25) # sparse solver gather tables (constant term products, CSC-ordered A) + branch-free A loads: parity, C5b / C5a / C2, C5b phase clocks
       $J "test:tests/test_netdes.py tests/test_sslp.py tests/test_bench_settings.py tests/test_gpu_parity.py" \
          "bench:r05_s25_c5b:--only C5b $A" "bench:r05_s25_c5a:--only C5a $A" "bench:r05_s25_c2:--only C2 $A" && \
       PHX_SP_PROF=1 $J "bench:r05_s25_c5b_spprof:--only C5b $A" ;;
  s26) # C4 with every timed launch bracketed; C5a workgroup round budget 6 / 8 against 4
       $J "bench:r05_s26_c4:--only C4 $A" "bench:r05_s26_c5a:--only C5a $A" \
          "bench:r05_s26_c5a_w6:--only C5a $A --so {\"wg_warm\":6}" "bench:r05_s26_c5a_w8:--only C5a $A --so {\"wg_warm\":8}" ;;
  s27) # the sparse solver's split level 2 (tv in the slot too: four workgroups per CU with the capped kernel) on C5b: parity, time
       PHX_SP_SPLIT=2 $J "test:tests/test_netdes.py" "bench:r05_s27_c5b_split2:--only C5b $A" && \
       $J "bench:r05_s27_c5b:--only C5b $A" ;;
  final) # the round's evidence: the whole GPU suite, the driver's default command, kernel traces
       $J "test:tests" && $J "py:r05_final_smoke:scripts/run_smoke.py" "bench:r05_final_default:--detail gpurun_out/r05_final_default_detail.json" \
          "prof:r05_final_prof:$H --ar-probe 0" "prof:r05_final_c3s8_prof:$S8" "prof:r05_final_1m_prof:$M" \
          "prof:r05_final_c2_prof:--only C2 $A" "prof:r05_final_c4_prof:--only C4 $A" "prof:r05_final_c5a_prof:--only C5a $A" \
          "prof:r05_final_c5b_prof:--only C5b $A" ;;
  pmc1) # PMC passes on the final kernels (one counter group per pass): the lane kernels
       $J "pmc:r05_pmc_c3_fetch:FETCH_SIZE:$B" "pmc:r05_pmc_c3_write:WRITE_SIZE:$B" "pmc:r05_pmc_c3_sq:$SQ:$B" \
          "pmc:r05_pmc_s8_fetch:FETCH_SIZE:$S8" "pmc:r05_pmc_s8_write:WRITE_SIZE:$S8" "pmc:r05_pmc_s8_sq:$SQ:$S8" \
          "pmc:r05_pmc_1m_fetch:FETCH_SIZE:$M" "pmc:r05_pmc_1m_write:WRITE_SIZE:$M" \
          "pmc:r05_pmc_c4_fetch:FETCH_SIZE:--only C4 $A" "pmc:r05_pmc_c4_write:WRITE_SIZE:--only C4 $A" ;;
  pmc2) # ... the workgroup and sparse solvers
       $J "pmc:r05_pmc_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r05_pmc_c2_write:WRITE_SIZE:--only C2 $A" \
          "pmc:r05_pmc_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r05_pmc_c5a_write:WRITE_SIZE:--only C5a $A" \
          "pmc:r05_pmc_c5b_fetch:FETCH_SIZE:--only C5b $A" "pmc:r05_pmc_c5b_write:WRITE_SIZE:--only C5b $A" ;;
  s28) # the workgroup pass's leftovers (the in-stream sparse interior point): C5a / C2 round budgets with single-change
       # rounds after a few full ones (PHX_WG_SINGLE_AFTER), sparse phase clocks for the leftovers' interior-point counts
       PHX_SP_PROF=1 $J "bench:r05_s28_c5a:--only C5a $A" "bench:r05_s28_c5a_w8:--only C5a $A --so {\"wg_warm\":8}" \
          "bench:r05_s28_c2:--only C2 $A" && \
       PHX_SP_PROF=1 PHX_WG_SINGLE_AFTER=4 $J "bench:r05_s28_c5a_w8_sa4:--only C5a $A --so {\"wg_warm\":8}" \
          "bench:r05_s28_c5a_w16_sa4:--only C5a $A --so {\"wg_warm\":16}" "bench:r05_s28_c2_sa4:--only C2 $A" \
          "bench:r05_s28_c2_w16_sa4:--only C2 $A --so {\"wg_warm\":16,\"wg_first\":1}" ;;
  s29) # sparse solver, small problems (sslp): every row / off-diagonal Schur entry / B row a quad -- parity, C5a / C5b / C2, clocks
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s29_c5a:--only C5a $A" "bench:r05_s29_c5b:--only C5b $A" "bench:r05_s29_c2:--only C2 $A" && \
       PHX_SP_PROF=1 $J "bench:r05_s29_c5a_spprof:--only C5a $A" ;;
  s30) # sparse solver: 1 / M_bb stored (multiplications in the Schur terms and the M solves) -- parity, C5a / C5b, clocks
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s30_c5a:--only C5a $A" "bench:r05_s30_c5b:--only C5b $A" && \
       PHX_SP_PROF=1 $J "bench:r05_s30_c5a_spprof:--only C5a $A" ;;
  s31) # (measured and reverted) the separator Schur term loops unrolled by four -- C5a / C5b, clocks
       $J "bench:r05_s31_c5a:--only C5a $A" "bench:r05_s31_c5b:--only C5b $A" && \
       PHX_SP_PROF=1 $J "bench:r05_s31_c5a_spprof:--only C5a $A" ;;
  s32) # headline solver-option sweep (same box): as_rounds 3 / 5 / 6 against 4, iterk depth 8, seed templates 32
       $J "bench:r05_s32_h:$H" "bench:r05_s32_h_as3:$H --so {\"as_rounds\":3}" "bench:r05_s32_h_as5:$H --so {\"as_rounds\":5}" \
          "bench:r05_s32_h_as6:$H --so {\"as_rounds\":6}" "bench:r05_s32_h_d8:$H --depth 8" \
          "bench:r05_s32_h_t32:$H --so {\"seed_templates\":32}" "bench:r05_s32_h2:$H" ;;
  s33) # the sparse scratch's row vectors in LDS (small problems): parity (incl. bit equality), C5a / C5b / C2, clocks
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s33_c5a:--only C5a $A" "bench:r05_s33_c5b:--only C5b $A" "bench:r05_s33_c2:--only C2 $A" && \
       PHX_SP_PROF=1 $J "bench:r05_s33_c5a_spprof:--only C5a $A" ;;
  s34) # the sparse scratch's column bounds shared when scenario-invariant: parity, C5a / C5b / C2
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s34_c5a:--only C5a $A" "bench:r05_s34_c5b:--only C5b $A" "bench:r05_s34_c2:--only C2 $A" ;;
  s35) # C5a: single-change workgroup rounds early (PHX_WG_SINGLE_AFTER) with larger budgets, against the default
       PHX_SP_PROF=1 $J "bench:r05_s35_c5a:--only C5a $A" && \
       PHX_SP_PROF=1 PHX_WG_SINGLE_AFTER=1 $J "bench:r05_s35_c5a_sa1_w16:--only C5a $A --so {\"wg_warm\":16}" \
          "bench:r05_s35_c5a_sa1_w32:--only C5a $A --so {\"wg_warm\":32}" && \
       PHX_SP_PROF=1 PHX_WG_SINGLE_AFTER=2 $J "bench:r05_s35_c5a_sa2_w16:--only C5a $A --so {\"wg_warm\":16}" && \
       PHX_SP_PROF=1 PHX_WG_SINGLE_AFTER=3 $J "bench:r05_s35_c5a_sa3_w24:--only C5a $A --so {\"wg_warm\":24}" ;;
  s36) # C4: the single-change rule (JIT defines): the multiplier first / the primal violation first, against the larger of the two
       $J "bench:r05_s36_c4:--only C4 $A" && PHX_LANE_DEFS="PHX_SINGLE_DUAL_FIRST" $J "bench:r05_s36_c4_dual:--only C4 $A" && \
       PHX_LANE_DEFS="PHX_SINGLE_PRIMAL_FIRST" $J "bench:r05_s36_c4_primal:--only C4 $A" && $J "bench:r05_s36_c4b:--only C4 $A" ;;
  s37) # (measured and reverted) the pivot pairs' divide / square-root chain formed one step ahead -- parity, C2 / C5a, clocks
       $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s37_c2:--only C2 $A" "bench:r05_s37_c5a:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s37_c2_wgprof:--only C2 $A" ;;
  s38) # the sparse interior point's loops with their loads ahead of the branches: parity, C5a / C5b / C2, clocks
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s38_c5a:--only C5a $A" "bench:r05_s38_c5b:--only C5b $A" "bench:r05_s38_c2:--only C2 $A" && \
       PHX_SP_PROF=1 $J "bench:r05_s38_c5a_spprof:--only C5a $A" ;;
  s39) # ... the same for the KKT error, classification and active-set rounds: parity, C5a / C5b / C2, clocks
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s39_c5a:--only C5a $A" "bench:r05_s39_c5b:--only C5b $A" "bench:r05_s39_c2:--only C2 $A" && \
       PHX_SP_PROF=1 $J "bench:r05_s39_c5b_spprof:--only C5b $A" ;;
  s40) # workgroup solver: operands loaded before branching in the refinement / certificate / update loops -- parity, C2 / C5a
       $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s40_c2:--only C2 $A" "bench:r05_s40_c5a:--only C5a $A" ;;
  s41) # refinement: the column residual after a step is reg dx (no recomputation, one barrier less per step) -- parity, C2 / C5a / C5b, clocks
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r05_s41_c2:--only C2 $A" "bench:r05_s41_c5a:--only C5a $A" "bench:r05_s41_c5b:--only C5b $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s41_c2_wgprof:--only C2 $A" ;;
  s42) # lane refinement: the column residual carried as reg d (PHX_REFINE_CARRY) -- the GPU suite under it, then A/B on one box
       PHX_LANE_DEFS=PHX_REFINE_CARRY $J "test:tests" && \
       $J "bench:r05_s42_bench:$H" && PHX_LANE_DEFS=PHX_REFINE_CARRY $J "bench:r05_s42_bench_carry:$H" && \
       $J "bench:r05_s42_1m:$M" && PHX_LANE_DEFS=PHX_REFINE_CARRY $J "bench:r05_s42_1m_carry:$M" && \
       $J "bench:r05_s42_c3s8:$S8" && PHX_LANE_DEFS=PHX_REFINE_CARRY $J "bench:r05_s42_c3s8_carry:$S8" && \
       $J "bench:r05_s42_c4:--only C4 $A" && PHX_LANE_DEFS=PHX_REFINE_CARRY $J "bench:r05_s42_c4_carry:--only C4 $A" && \
       $J "bench:r05_s42_bench2:$H" && PHX_LANE_DEFS=PHX_REFINE_CARRY $J "bench:r05_s42_bench_carry2:$H" ;;
  s43) # carried refinement residual by default except in the two-wave fused build -- the GPU suite, then A/B against PHX_REFINE_RECOMPUTE
       $J "test:tests" && \
       $J "bench:r05_s43_bench:$H" && PHX_LANE_DEFS=PHX_REFINE_RECOMPUTE $J "bench:r05_s43_bench_rc:$H" && \
       $J "bench:r05_s43_bench2:$H" && PHX_LANE_DEFS=PHX_REFINE_RECOMPUTE $J "bench:r05_s43_bench_rc2:$H" && \
       $J "bench:r05_s43_1m:$M" && PHX_LANE_DEFS=PHX_REFINE_RECOMPUTE $J "bench:r05_s43_1m_rc:$M" && \
       $J "bench:r05_s43_c3s8:$S8" "bench:r05_s43_c4:--only C4 $A" ;;
  s44) # workgroup / sparse cross-lane sums and maxes by DPP instead of ds_bpermute shuffles -- parity, C2 / C5a / C5b, clocks
       $J "test:tests/test_sslp.py tests/test_netdes.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py tests/test_wg_blk.py" \
          "bench:r05_s44_c2:--only C2 $A" "bench:r05_s44_c5a:--only C5a $A" "bench:r05_s44_c5b:--only C5b $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s44_c2_wgprof:--only C2 $A" ;;
  s45) # workgroup Cholesky: thread groups per trailing row as wide as the rows left allow -- parity, C2 / C5a, clocks
       $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py tests/test_wg_blk.py" \
          "bench:r05_s45_c2:--only C2 $A" "bench:r05_s45_c5a:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s45_c2_wgprof:--only C2 $A" ;;
  s46) # the sparse interior point's stopping tolerance (ipm_tol; the classification follows it): C5b / C5a Iter0 and step
       $J "bench:r05_s46_c5b:--only C5b $A" "bench:r05_s46_c5b_t8:--only C5b $A --so {\"ipm_tol\":1e-8}" \
          "bench:r05_s46_c5b_t6:--only C5b $A --so {\"ipm_tol\":1e-6}" \
          "bench:r05_s46_c5a:--only C5a $A" "bench:r05_s46_c5a_t8:--only C5a $A --so {\"ipm_tol\":1e-8}" \
          "bench:r05_s46_c5a_t6:--only C5a $A --so {\"ipm_tol\":1e-6}" ;;
  s47) # Iter0 bookkeeping with batched loads and a parallel fold; the fused loop's last copies stored by its tail kernel
       $J "test:tests" && $J "bench:r05_s47_bench:$H" "bench:r05_s47_bench2:$H" "bench:r05_s47_1m:$M" "bench:r05_s47_c3s8:$S8" \
          "prof:r05_s47_prof:$H --ar-probe 0" ;;
  s48) # workgroup refinement: thread groups per active row / factor row as wide as the active rows allow (DPP group
       # sums) -- measured slower (rows / solve clocks 199 / 210 -> 215 / 231 Mcycles) and reverted
       $J "test:tests/test_sslp.py tests/test_bench_settings.py tests/test_trajectories.py tests/test_gpu_parity.py tests/test_wg_blk.py" \
          "bench:r05_s48_c2:--only C2 $A" "bench:r05_s48_c5a:--only C5a $A" "bench:r05_s48_c2b:--only C2 $A" && \
       PHX_WG_PROF=1 $J "bench:r05_s48_c2_wgprof:--only C2 $A" ;;
  s49) # deferred Iter0 without statistics / completion markers (ev_run recorded at the finish; adoption needs none)
       $J "test:tests" && $J "bench:r05_s49_bench:$H" "bench:r05_s49_bench2:$H" "bench:r05_s49_c3s8:$S8" \
          "prof:r05_s49_prof:$H --ar-probe 0" ;;
  s50) # Iter0's pass counts stored into mapped host memory by a small kernel instead of a blit copy -- the same time
       # (the kernel 4.5 us, then the same 5.8 us gap before the next: the host-memory writes' release), reverted
       $J "test:tests" && $J "bench:r05_s50_bench:$H" "bench:r05_s50_bench2:$H" "prof:r05_s50_prof:$H --ar-probe 0" ;;
  s51) # the timed object built before the warmup (the warmup's steps right before the timed region) against after it
       $J "bench:r05_s51_new1:$H" "bench:r05_s51_old1:$H --build-after-warmup" "bench:r05_s51_new2:$H" \
          "bench:r05_s51_old2:$H --build-after-warmup" "bench:r05_s51_new3:$H" "bench:r05_s51_old3:$H --build-after-warmup" ;;
  s52) # final evidence on the final sources: the whole GPU suite, then the driver's default command
       $J "test:tests" && $J "bench:r05_s52_default:--detail gpurun_out/r05_s52_default_detail.json" ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
