#!/bin/bash
# Round-3 GPU evidence jobs (run through gpurun): bash scripts/jobs_r03.sh <name>.
# Each job is a list of scripts/gpu_job.sh steps; logs land in gpurun_out/, the
# summaries judged are copied into profiles/ (named after the job).
set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"                 # headline, K = 50
H="--configs none --no-cpu-baseline --no-conv"                            # headline, K = 20 (driver shape)
M="--configs none --no-cpu-baseline --no-conv --steps 20 --warmup 1 --scens 1000000 --ar-probe 0"   # over-cache 1M
A="--no-cpu-baseline --no-conv --steps 10 --warmup 1"                     # one secondary config
SQ="SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU_FLOPS_FP64,SQ_INSTS_SALU"
J="bash scripts/gpu_job.sh"
case "$1" in
  s1)  $J "test:tests" "bench:r03_s1_bench:$H" ;;
  s2)  $J "trace:r03_s2_trace:$H --ar-probe 0" "prof:r03_s2_prof:$H --ar-probe 0" ;;
  s3)  $J "test:tests/test_gpu_parity.py -k factor_cache" "bench:r03_s3_c2:--only C2 $A" \
          "trace:r03_s3_trace:$H --ar-probe 0" ;;
  s4)  $J "test:tests/test_gpu_parity.py -k deferred_iter0" "test:tests" "bench:r03_s4_bench:$H" \
          "trace:r03_s4_trace:$H --ar-probe 0" ;;
  s5)  $J "test:tests/test_gpu_parity.py tests/test_hydro.py" "bench:r03_s5_bench:$H" \
          "trace:r03_s5_trace:$H --ar-probe 0" ;;
  s6)  $J "test:tests/test_gpu_parity.py tests/test_hydro.py" "bench:r03_s6_bench:$H" \
          "bench:r03_s6_bench_noseed:$H --so {\"seed_templates\":0}" \
          "trace:r03_s6_trace:$H --ar-probe 0" "trace:r03_s6_trace_noseed:$H --ar-probe 0 --so {\"seed_templates\":0}" ;;
  s7)  $J "py:r03_s7_host_marks:scripts/host_marks.py 100000 20 5" "bench:r03_s7_c2:--only C2 $A" ;;
  s8)  $J "test:tests/test_gpu_parity.py tests/test_hydro.py" "bench:r03_s8_bench:$H" \
          "trace:r03_s8_trace:$H --ar-probe 0" "py:r03_s8_host_marks:scripts/host_marks.py 100000 20 5" && \
       PHX_LANE_STAMPS=1 $J "bench:r03_s8_stamps:$H --ar-probe 0" ;;
  s9)  $J "trace:r03_s9_trace_unfused:$H --ar-probe 0 --fused 0" && \
       PHX_FRESH_LIST=1 $J "trace:r03_s9_trace_unfused_list:$H --ar-probe 0 --fused 0" ;;
  s10) $J "test:tests/test_sslp.py tests/test_trajectories.py tests/test_gpu_parity.py::test_sslp_ph_gpu tests/test_gpu_parity.py::test_sslp_synthetic_batch_gpu tests/test_gpu_parity.py::test_farmer_cm10_1000_workgroup_gpu tests/test_gpu_parity.py::test_native_loop_workgroup_matches_host_loop_gpu tests/test_gpu_parity.py::test_native_loop_workgroup_stragglers_gpu tests/test_gpu_parity.py::test_wg_factor_cache_gpu" \
          "bench:r03_s10_c2:--only C2 $A" "bench:r03_s10_c5a:--only C5a $A" \
          "trace:r03_s9_trace_unfused:$H --ar-probe 0 --fused 0" && \
       PHX_FRESH_LIST=1 $J "trace:r03_s9_trace_unfused_list:$H --ar-probe 0 --fused 0" ;;
  s11) $J "test:tests" "bench:r03_s11_bench:$H" "trace:r03_s11_trace:$H --ar-probe 0" ;;
  s12) $J "test:tests" "bench:r03_s12_bench:$H" "trace:r03_s12_trace:$H --ar-probe 0" \
          "bench:r03_s12_c5b:--only C5b $A" ;;
  s13) PHX_WG_PROF=1 $J "bench:r03_s13_c2_wgprof:--only C2 $A --so {\"native_loop\":0}" && \
       PHX_SP_GRID=64 $J "bench:r03_s13_c5b_g64:--only C5b $A" && PHX_SP_GRID=128 $J "bench:r03_s13_c5b_g128:--only C5b $A" ;;
  s14) $J "test:tests" "bench:r03_s14_bench:$H" "trace:r03_s14_trace:$H --ar-probe 0" && \
       PHX_WG_PROF=1 $J "bench:r03_s13_c2_wgprof:--only C2 $A --so {\"native_loop\":0}" && \
       PHX_SP_GRID=64 $J "bench:r03_s13_c5b_g64:--only C5b $A" && PHX_SP_GRID=128 $J "bench:r03_s13_c5b_g128:--only C5b $A" ;;
  s15) $J "test:tests" "bench:r03_s15_bench_default:" "prof:r03_s15_prof:$B" \
          "pmc:r03_s15_pmc_fetch:FETCH_SIZE:$B" "pmc:r03_s15_pmc_write:WRITE_SIZE:$B" "pmc:r03_s15_pmc_sq:$SQ:$B" ;;
  s16) $J "pmc:r03_s16_pmc1m_fetch:FETCH_SIZE:$M" "pmc:r03_s16_pmc1m_write:WRITE_SIZE:$M" \
          "pmc:r03_s16_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r03_s16_c2_write:WRITE_SIZE:--only C2 $A" \
          "pmc:r03_s16_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r03_s16_c5a_write:WRITE_SIZE:--only C5a $A" \
          "pmc:r03_s16_c5b_fetch:FETCH_SIZE:--only C5b $A" "pmc:r03_s16_c5b_write:WRITE_SIZE:--only C5b $A" ;;
  s17) $J "test:tests/test_prox_approx.py tests/test_cylinders.py tests/test_abi_layout.py tests/test_gpu_parity.py" \
          "bench:r03_s17_c2:--only C2 $A" "bench:r03_s17_c5a:--only C5a $A" \
          "pmc:r03_s17_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r03_s17_c2_write:WRITE_SIZE:--only C2 $A" \
          "pmc:r03_s17_c5a_write:WRITE_SIZE:--only C5a $A" ;;
  s18) $J "test:tests" "bench:r03_s18_bench_default:" "prof:r03_s18_prof:$H --ar-probe 0" ;;
  s19) $J "test:tests/test_netdes.py tests/test_sslp.py tests/test_trajectories.py" \
          "bench:r03_s19_c5b_split:--only C5b $A" && PHX_SP_SPLIT=0 $J "bench:r03_s19_c5b_nosplit:--only C5b $A" ;;
  s20) $J "pmc:r03_s20_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r03_s20_c5a_write:WRITE_SIZE:--only C5a $A" \
          "pmc:r03_s20_c5b_fetch:FETCH_SIZE:--only C5b $A" "pmc:r03_s20_c5b_write:WRITE_SIZE:--only C5b $A" \
          "pmc:r03_s20_c4_fetch:FETCH_SIZE:--only C4 $A" "pmc:r03_s20_c4_write:WRITE_SIZE:--only C4 $A" ;;
  s21) $J "test:tests/test_sslp.py tests/test_gpu_parity.py tests/test_trajectories.py" \
          "bench:r03_s21_c5a_split:--only C5a $A" "bench:r03_s21_c2:--only C2 $A" && \
       PHX_WG_SPLIT=0 $J "bench:r03_s21_c5a_nosplit:--only C5a $A" ;;
  s22) $J "bench:r03_s22_base1:$H --ar-probe 0" "bench:r03_s22_base50:$B --ar-probe 0" && \
       PHX_LANE_DEFS=PHX_OUT_WT $J "bench:r03_s22_wt1:$H --ar-probe 0" "bench:r03_s22_wt50:$B --ar-probe 0" \
          "prof:r03_s22_wt_prof:$H --ar-probe 0" && \
       $J "bench:r03_s22_base2:$H --ar-probe 0" && PHX_LANE_DEFS=PHX_OUT_WT $J "bench:r03_s22_wt2:$H --ar-probe 0" ;;
  s23) $J "test:tests" "bench:r03_s23_bench_default:" "prof:r03_s23_prof:$H --ar-probe 0" \
          "pmc:r03_s23_pmc_fetch:FETCH_SIZE:$B" "pmc:r03_s23_pmc_write:WRITE_SIZE:$B" "pmc:r03_s23_pmc_sq:$SQ:$B" ;;
  s24) $J "test:tests/test_netdes.py tests/test_sslp.py tests/test_trajectories.py tests/test_gpu_parity.py" \
          "bench:r03_s24_c2:--only C2 $A" "bench:r03_s24_c5b:--only C5b $A" "bench:r03_s24_c5a:--only C5a $A" ;;
  s25) $J "prof:r03_s25_c2_prof:--only C2 $A" ;;
  s26) $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_hydro.py" \
          "bench:r03_s26_c2:--only C2 $A" "bench:r03_s26_c4:--only C4 $A" "prof:r03_s26_c2_prof:--only C2 $A" ;;
  s27) $J "test:tests" "bench:r03_s27_bench_default:" "prof:r03_s27_c2_prof:--only C2 $A" ;;
  s28) $J "test:tests/test_gpu_parity.py tests/test_trajectories.py tests/test_prox_approx.py tests/test_sslp.py" \
          "bench:r03_s28_c2:--only C2 $A" "bench:r03_s28_c4:--only C4 $A" "bench:r03_s28_c5a:--only C5a $A" "prof:r03_s28_c2_prof:--only C2 $A" ;;
  s29) $J "test:tests/test_netdes.py tests/test_sslp.py tests/test_gpu_parity.py tests/test_trajectories.py" \
          "bench:r03_s29_c5b:--only C5b $A" "bench:r03_s29_c2:--only C2 $A" "bench:r03_s29_c5a:--only C5a $A" ;;
  s30) $J "test:tests" "bench:r03_s30_bench_default:" ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
