#!/bin/bash
# Round-4 GPU evidence jobs (run through gpurun): bash scripts/jobs_r04.sh <name>.
# Each job is a list of scripts/gpu_job.sh steps; logs land in gpurun_out/, the
# summaries judged are copied into profiles/ (named after the job).
set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"                 # headline, K = 50
H="--configs none --no-cpu-baseline --no-conv"                            # headline, K = 20 (driver shape)
M="--configs none --no-cpu-baseline --no-conv --steps 20 --warmup 1 --scens 1000000 --ar-probe 0"   # over-cache 1M
A="--no-cpu-baseline --no-conv --steps 10 --warmup 1"                     # one secondary config
S8="--only C3s8 --no-cpu-baseline --no-conv --steps 20"                   # the 8-GPU per-rank slice
SQ="SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU_FLOPS_FP64,SQ_INSTS_SALU"
J="bash scripts/gpu_job.sh"
case "$1" in
  s1)  $J "bench:r04_s1_c3s8:$S8" "prof:r04_s1_c3s8_prof:$S8" "prof:r04_s1_prof:$H --ar-probe 0" && \
       PHX_LANE_STAMPS=1 $J "bench:r04_s1_c3s8_stamps:$S8" ;;
  s2)  $J "test:tests" "bench:r04_s2_c3s8:$S8" "bench:r04_s2_bench:$H" "prof:r04_s2_c3s8_prof:$S8" && \
       PHX_LANE_DEFS=PHX_RELAXED_HANDOFF $J "bench:r04_s2_bench_relaxed:$H" "bench:r04_s2_c3s8_relaxed:$S8" ;;
  s3)  $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py" "bench:r04_s3_c3s8:$S8" \
          "bench:r04_s3_bench:$H" "prof:r04_s3_prof:$H --ar-probe 0" "prof:r04_s3_c3s8_prof:$S8" && \
       PHX_LANE_STAMPS=1 $J "bench:r04_s3_c3s8_stamps:$S8" "bench:r04_s3_stamps:$H --ar-probe 0" ;;
  s4)  $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py tests/test_engine_emu.py" \
          "bench:r04_s4_c3s8:$S8" "bench:r04_s4_bench:$H" "prof:r04_s4_prof:$H --ar-probe 0" "prof:r04_s4_c3s8_prof:$S8" && \
       PHX_FZ_LEGACY=1 $J "bench:r04_s4_c3s8_legacy:$S8" "bench:r04_s4_bench_legacy:$H" && \
       PHX_LANE_STAMPS=1 $J "bench:r04_s4_c3s8_stamps:$S8" "bench:r04_s4_stamps:$H --ar-probe 0" ;;
  s5)  # the workgroup solver's factor cache, pay or drop; its phase clocks; the default command
       $J "bench:r04_s5_c2:--only C2 $A" "bench:r04_s5_c5a:--only C5a $A" "prof:r04_s5_c4_prof:--only C4 $A" && \
       PHX_WG_NO_FACTOR_CACHE=1 $J "bench:r04_s5_c2_nocache:--only C2 $A" "bench:r04_s5_c5a_nocache:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r04_s5_c2_wgprof:--only C2 $A" "bench:r04_s5_c5a_wgprof:--only C5a $A" && \
       $J "bench:r04_s5_default:" ;;
  s6)  # host launch calls against device starts (the loop's dispatch gaps)
       $J "trace:r04_s6_c3s8_trace:$S8" "trace:r04_s6_trace:$H --ar-probe 0" ;;
  s7)  # the poll without stream queries: the fused loop's dispatch gaps
       $J "bench:r04_s7_c3s8:$S8" "bench:r04_s7_bench:$H" "trace:r04_s7_c3s8_trace:$S8" "trace:r04_s7_trace:$H --ar-probe 0" ;;
  s8)  # window timing of the fused launches (no event records inside the loop)
       $J "test:tests/test_gpu_parity.py -k window_timing" "bench:r04_s8_c3s8:$S8" "bench:r04_s8_bench:$H" \
          "prof:r04_s8_c3s8_prof:$S8" "prof:r04_s8_prof:$H --ar-probe 0" ;;
  s9)  # the workgroup solver's phase clocks in the device loop
       PHX_WG_PROF=1 $J "bench:r04_s9_c2_wgprof:--only C2 $A" "bench:r04_s9_c5a_wgprof:--only C5a $A" ;;
  s10) # the 1M configuration's loop (r04 s5: 10.9 ms per iteration, unfused)
       PHX_ITERK_DEBUG=1 $J "bench:r04_s10_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       PHX_QUERY_MS=0 $J "bench:r04_s10_1m_q0:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" ;;
  s11) # the blocked MFMA Schur inverse in the workgroup solver: tests, C2 / C5a with and without, phase clocks
       $J "test:tests/test_wg_blk.py tests/test_sslp.py tests/test_bundles.py tests/test_trajectories.py" \
          "bench:r04_s11_c2:--only C2 $A" "bench:r04_s11_c5a:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r04_s11_c2_wgprof:--only C2 $A" "bench:r04_s11_c5a_wgprof:--only C5a $A" && \
       PHX_WG_BLK=0 $J "bench:r04_s11_c2_scalar:--only C2 $A" "bench:r04_s11_c5a_scalar:--only C5a $A" ;;
  s12) # workgroup solver modes: blocked factor + inverse (default), + X^T X, scalar
       $J "test:tests/test_wg_blk.py tests/test_sslp.py tests/test_bundles.py tests/test_trajectories.py" \
          "bench:r04_s12_c2:--only C2 $A" "bench:r04_s12_c5a:--only C5a $A" && \
       PHX_WG_PROF=1 $J "bench:r04_s12_c2_wgprof:--only C2 $A" "bench:r04_s12_c5a_wgprof:--only C5a $A" && \
       PHX_WG_BLK=2 $J "bench:r04_s12_c2_blk2:--only C2 $A" "bench:r04_s12_c5a_blk2:--only C5a $A" && \
       PHX_WG_BLK=0 $J "bench:r04_s12_c2_scalar:--only C2 $A" "bench:r04_s12_c5a_scalar:--only C5a $A" ;;
  s13) # the 1M loop's straggler stops: fused kernel vs the legacy fused launch
       $J "bench:r04_s13_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       PHX_FZ_LEGACY=1 $J "bench:r04_s13_1m_legacy:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" ;;
  s14) # the 1M loop's kernel trace
       $J "prof:r04_s14_1m_prof:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" ;;
  s15) # the 1M configuration after the cold-path fixes; the per-rank slice's profile
       $J "bench:r04_s15_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" \
          "bench:r04_s15_c3s8:$S8" "prof:r04_s15_c3s8_prof:$S8" "bench:r04_s15_bench:$H" ;;
  s16) # the 100k Iter0: unseeded (interior point on every lane) against seeded
       $J "bench:r04_s16_bench:$H" && PHX_NO_SEED=1 $J "bench:r04_s16_bench_noseed:$H" "prof:r04_s16_noseed_prof:$H --ar-probe 0" ;;
  s17) # the 1M Iter0: unseeded against seeded
       $J "bench:r04_s17_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       PHX_NO_SEED=1 $J "bench:r04_s17_1m_noseed:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" ;;
  s18) # the whole GPU suite, then the driver's default command
       $J "test:tests" && $J "bench:r04_s18_default:" ;;
  s19) # the workgroup solver's pipeline stops (C5a, C2 traces) with single changes after two rounds, and without
       $J "prof:r04_s19_c5a_prof:--only C5a $A" "bench:r04_s19_c5a:--only C5a $A" "bench:r04_s19_c2:--only C2 $A" && \
       PHX_WG_SINGLE_AFTER=99 $J "bench:r04_s19_c5a_full:--only C5a $A" "bench:r04_s19_c2_full:--only C2 $A" ;;
  s20) # the sparse solver's factorization share: every factorization done twice (variant build)
       $J "bench:r04_s20_c5b:--only C5b $A" "bench:r04_s20_c5a:--only C5a $A" "bench:r04_s20_c2:--only C2 $A" && \
       PHX_LIB_PATH=$PWD/mpi-sppy_amd/libphx_sptwice.so $J "bench:r04_s20_c5b_twice:--only C5b $A" \
          "bench:r04_s20_c5a_twice:--only C5a $A" "bench:r04_s20_c2_twice:--only C2 $A" ;;
  s21) # the factor's and the refinement's shares of the lane round (JIT measurement defines)
       $J "bench:r04_s21_c3s8:$S8" "bench:r04_s21_bench:$H" && \
       PHX_LANE_DEFS=PHX_EXP_FACTOR_TWICE $J "bench:r04_s21_c3s8_f2:$S8" "bench:r04_s21_bench_f2:$H" && \
       PHX_LANE_DEFS=PHX_EXP_REFINE_TWICE $J "bench:r04_s21_c3s8_r2:$S8" "bench:r04_s21_bench_r2:$H" ;;
  s22) # the one-wave fused kernel's rounds on register data (no per-round re-load)
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py" "bench:r04_s22_c3s8:$S8" "prof:r04_s22_c3s8_prof:$S8" && \
       PHX_LANE_DEFS=PHX_FZ1_RELOAD $J "bench:r04_s22_c3s8_reload:$S8" ;;
  s23) # the one-wave fused kernel at 100k and 1M (waves one after the other on a SIMD)
       $J "bench:r04_s23_bench:$H" "bench:r04_s23_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       PHX_FZ1=1 $J "bench:r04_s23_bench_fz1:$H" "bench:r04_s23_1m_fz1:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" ;;
  s24) # the one-wave fused kernel at 1M: HBM traffic and time again
       PHX_FZ1=1 $J "pmc:r04_s24_1m_fz1_fetch:FETCH_SIZE:$M" "pmc:r04_s24_1m_fz1_write:WRITE_SIZE:$M" \
          "bench:r04_s24_1m_fz1:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       $J "bench:r04_s24_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" ;;
  s25) # the one-wave fused kernel at 100k: traffic, and time against the two-wave build twice
       PHX_FZ1=1 $J "pmc:r04_s25_c3_fz1_fetch:FETCH_SIZE:$B" "pmc:r04_s25_c3_fz1_write:WRITE_SIZE:$B" \
          "bench:r04_s25_bench_fz1a:$H" && $J "bench:r04_s25_bencha:$H" && PHX_FZ1=1 $J "bench:r04_s25_bench_fz1b:$H" && \
       $J "bench:r04_s25_benchb:$H" ;;
  s26) # phx_lane_all with the interior point out of line; the single-change rule (C4, C3s8)
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py" "bench:r04_s26_c4:--only C4 $A" \
          "prof:r04_s26_c4_prof:--only C4 $A" "bench:r04_s26_c3s8:$S8" && \
       PHX_LANE_DEFS=PHX_ALL_INLINE $J "bench:r04_s26_c4_inline:--only C4 $A" "bench:r04_s26_c3s8_inline:$S8" && \
       PHX_LANE_DEFS=PHX_SINGLE_LARGEST $J "bench:r04_s26_c4_largest:--only C4 $A" "bench:r04_s26_c3s8_largest:$S8" && \
       PHX_LANE_DEFS=PHX_SINGLE_DUAL_FIRST $J "bench:r04_s26_c4_dual:--only C4 $A" "bench:r04_s26_c3s8_dual:$S8" ;;
  s27) # the loop's tail: copies enqueued with the last iteration, lazy counter resets; host wall timelines
       $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py tests/test_engine_emu.py" \
          "bench:r04_s27_c3s8:$S8" "bench:r04_s27_bench:$H" "prof:r04_s27_c3s8_prof:$S8" && \
       SCENS=12500 timeout -k 10 200 python scripts/iter0_wall.py > gpurun_out/r04_s27_wall_12k5.txt 2>&1 && \
       SCENS=100000 timeout -k 10 200 python scripts/iter0_wall.py > gpurun_out/r04_s27_wall_100k.txt 2>&1 && \
       $J "bench:r04_s27_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       PHX_LANE_DEFS=PHX_LIST_RELOAD $J "bench:r04_s27_bench_reload:$H" \
          "bench:r04_s27_1m_reload:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       $J "bench:r04_s27_c4:--only C4 $A" "prof:r04_s27_c4_prof:--only C4 $A" && \
       PHX_LANE_DEFS=PHX_ALL_RELOAD $J "bench:r04_s27_c3s8_allreload:$S8" "bench:r04_s27_c4_allreload:--only C4 $A" ;;
  s28) # Iter0's E1 sum at construction (host)
       $J "test:tests/test_gpu_parity.py tests/test_engine_emu.py" "bench:r04_s28_bench:$H" "bench:r04_s28_c3s8:$S8" \
          "bench:r04_s28_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" ;;
  s29) # small batches: phx_lane_all against the separate passes (warm, register-resident rescue list, cold)
       $J "bench:r04_s29_c4:--only C4 $A" "bench:r04_s29_c3s8:$S8" && \
       PHX_NO_ALL=1 $J "bench:r04_s29_c4_noall:--only C4 $A" "bench:r04_s29_c3s8_noall:$S8" "prof:r04_s29_c4_noall_prof:--only C4 $A" && \
       $J "bench:r04_s29_c4b:--only C4 $A" && PHX_NO_ALL=1 $J "bench:r04_s29_c4b_noall:--only C4 $A" ;;
  s30) # the warm pass at one wave per SIMD with register-resident rounds (PHX_WARM_REG), A/B twice
       $J "bench:r04_s30_bench:$H" && PHX_LANE_DEFS=PHX_WARM_REG $J "bench:r04_s30_bench_wreg:$H" \
          "bench:r04_s30_1m_wreg:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       $J "bench:r04_s30_bench2:$H" "bench:r04_s30_1m:--only C3x1M --no-cpu-baseline --no-conv --steps 10 --warmup 1" && \
       PHX_LANE_DEFS=PHX_WARM_REG $J "bench:r04_s30_bench_wreg2:$H" ;;
  s31) # workgroup round budgets: C5a (config default 4) and C2 (library default 16)
       $J "bench:r04_s31_c5a_w3:--only C5a $A --so {\"wg_warm\":3}" "bench:r04_s31_c5a_w4:--only C5a $A" \
          "bench:r04_s31_c5a_w6:--only C5a $A --so {\"wg_warm\":6}" "bench:r04_s31_c2_w8:--only C2 $A --so {\"wg_warm\":8}" \
          "bench:r04_s31_c2_w16:--only C2 $A" "bench:r04_s31_c2_w24:--only C2 $A --so {\"wg_warm\":24}" ;;
  s32) # C2 round budget again (noise) and below
       $J "bench:r04_s32_c2_w4:--only C2 $A --so {\"wg_warm\":4}" "bench:r04_s32_c2_w6:--only C2 $A --so {\"wg_warm\":6}" \
          "bench:r04_s32_c2_w8:--only C2 $A --so {\"wg_warm\":8}" "bench:r04_s32_c2_w16:--only C2 $A" \
          "bench:r04_s32_c2_w8b:--only C2 $A --so {\"wg_warm\":8}" "bench:r04_s32_c2_w16b:--only C2 $A" ;;
  final) # the round's evidence: the whole GPU suite, the driver's default command, kernel traces
       $J "test:tests" && $J "bench:r04_final_default:" "prof:r04_final_prof:$H --ar-probe 0" \
          "prof:r04_final_c3s8_prof:$S8" "prof:r04_final_1m_prof:$M" "prof:r04_final_c2_prof:--only C2 $A" \
          "prof:r04_final_c4_prof:--only C4 $A" "prof:r04_final_c5a_prof:--only C5a $A" "prof:r04_final_c5b_prof:--only C5b $A" ;;
  pmc1) # PMC passes on the final kernels (one counter group per pass): the lane kernels
       $J "pmc:r04_pmc_c3_fetch:FETCH_SIZE:$B" "pmc:r04_pmc_c3_write:WRITE_SIZE:$B" "pmc:r04_pmc_c3_sq:$SQ:$B" \
          "pmc:r04_pmc_s8_fetch:FETCH_SIZE:$S8" "pmc:r04_pmc_s8_write:WRITE_SIZE:$S8" "pmc:r04_pmc_s8_sq:$SQ:$S8" \
          "pmc:r04_pmc_1m_fetch:FETCH_SIZE:$M" "pmc:r04_pmc_1m_write:WRITE_SIZE:$M" \
          "pmc:r04_pmc_c4_fetch:FETCH_SIZE:--only C4 $A" "pmc:r04_pmc_c4_write:WRITE_SIZE:--only C4 $A" ;;
  pmc2) # ... the workgroup and sparse solvers
       $J "pmc:r04_pmc_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r04_pmc_c2_write:WRITE_SIZE:--only C2 $A" \
          "pmc:r04_pmc_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r04_pmc_c5a_write:WRITE_SIZE:--only C5a $A" \
          "pmc:r04_pmc_c5b_fetch:FETCH_SIZE:--only C5b $A" "pmc:r04_pmc_c5b_write:WRITE_SIZE:--only C5b $A" ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
