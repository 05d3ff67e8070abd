#!/bin/bash
# Round-2 GPU evidence jobs (run through gpurun): bash scripts/jobs_r02.sh <name>.
# Each job is a list of scripts/gpu_job.sh steps; logs land in gpurun_out/, the
# summaries judged are copied into profiles/ (named after the job).
set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"                 # headline, K = 50
M="--configs none --no-cpu-baseline --no-conv --steps 20 --warmup 1 --scens 1000000"   # over-cache 1M
A="--no-cpu-baseline --no-conv --steps 10 --warmup 1"                     # one secondary config
SQ="SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU_FLOPS_FP64,SQ_INSTS_SALU"
J="bash scripts/gpu_job.sh"
case "$1" in
  s8)  $J "test:tests" "bench:r02_s8_bench:" "prof:r02_s8_prof:$B" "pmc:r02_s8_pmc_fetch:FETCH_SIZE:$B" \
          "pmc:r02_s8_pmc_write:WRITE_SIZE:$B" "pmc:r02_s8_pmc_sq:$SQ:$B" ;;
  s9)  $J "test:tests/test_gpu_parity.py -k workgroup" "bench:r02_s9_c2:--only C2 $A" "bench:r02_s9_w2:$B" \
       && PHX_LANE_WAVES=1 $J "bench:r02_s9_w1:$B" \
       && $J "bench:r02_s9_1m:$M" "pmc:r02_s9_pmc1m_fetch:FETCH_SIZE:$M" "pmc:r02_s9_pmc1m_write:WRITE_SIZE:$M" ;;
  s10) $J "test:tests" "bench:r02_s10_bench:" "prof:r02_s10_prof:$B" "pmc:r02_s10_pmc_fetch:FETCH_SIZE:$B" \
          "pmc:r02_s10_pmc_write:WRITE_SIZE:$B" ;;
  s11) $J "py:r02_s11_first:scripts/probe_first.py" "py:r02_s11_wall:scripts/iter0_wall.py" \
          "bench:r02_s11_c5b:--only C5b $A" "pmc:r02_s11_c5b_fetch:FETCH_SIZE:--only C5b $A" \
          "pmc:r02_s11_c5b_write:WRITE_SIZE:--only C5b $A" ;;
  s12) $J "pmc:r02_s12_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r02_s12_c2_write:WRITE_SIZE:--only C2 $A" \
          "pmc:r02_s12_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r02_s12_c5a_write:WRITE_SIZE:--only C5a $A" \
          "pmc:r02_s12_c4_fetch:FETCH_SIZE:--only C4 $A" "pmc:r02_s12_c4_write:WRITE_SIZE:--only C4 $A" ;;
  s13) $J "py:r02_s13_hostops:scripts/probe_host_ops.py" "bench:r02_s13_bench:--configs none --no-cpu-baseline --no-conv" \
          "py:r02_s13_wall:scripts/iter0_wall.py" ;;
  s14) $J "py:r02_s14_wall:scripts/iter0_wall.py" ;;
  s15) $J "py:r02_s15_hostops:scripts/probe_host_ops.py" ;;
  s16) $J "py:r02_s16_c2loop:scripts/probe_c2_loop.py" "trace:r02_s16_c2trace:--only C2 --no-cpu-baseline --no-conv --steps 20 --warmup 1" ;;
  s17) $J "test:tests/test_gpu_parity.py tests/test_sslp.py tests/test_netdes.py" "py:r02_s17_c2loop:scripts/probe_c2_loop.py" \
          "bench:r02_s17_c5a:--only C5a $A" ;;
  s18) $J "py:r02_s18_wgrounds:scripts/probe_wg_rounds.py" ;;
  s19) $J "py:r02_s19_smoke:scripts/run_smoke.py" "test:tests" "bench:r02_s19_bench:" "prof:r02_s19_prof:$B" ;;
  s20) $J "bench:r02_s20_bench:--configs none --no-cpu-baseline --no-conv" "pmc:r02_s20_pmc_sq:$SQ:$B" \
          "bench:r02_s20_1m:$M" "pmc:r02_s20_pmc1m_fetch:FETCH_SIZE:$M" "pmc:r02_s20_pmc1m_write:WRITE_SIZE:$M" \
          "pmc:r02_s20_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r02_s20_c5a_write:WRITE_SIZE:--only C5a $A" ;;
  s21) $J "test:tests" "bench:r02_s21_bench:--configs none --no-cpu-baseline --no-conv" "py:r02_s21_wall:scripts/iter0_wall.py" ;;
  s22) $J "py:r02_s22_smoke:scripts/run_smoke.py" "bench:r02_s22_bench:" ;;
  s23) $J "test:tests/test_gpu_parity.py" "bench:r02_s23_bench:--configs none --no-cpu-baseline --no-conv" \
          "bench:r02_s23_bench_b:--configs none --no-cpu-baseline --no-conv" ;;
  s24) $J "test:tests" "bench:r02_s24_bench:--configs none --no-cpu-baseline --no-conv" \
          "prof:r02_s24_prof:$B" "pmc:r02_s24_pmc_fetch:FETCH_SIZE:$B" "pmc:r02_s24_pmc_write:WRITE_SIZE:$B" ;;
  s25) $J "bench:r02_s25_1m:$M" "pmc:r02_s25_pmc1m_fetch:FETCH_SIZE:$M" "pmc:r02_s25_pmc1m_write:WRITE_SIZE:$M" ;;
  s26) $J "prof:r02_s26_c2_prof:--only C2 $A" "prof:r02_s26_c5a_prof:--only C5a $A" "prof:r02_s26_c5b_prof:--only C5b $A" ;;
  *) echo "usage: $0 s8|s9|...|s20"; exit 2 ;;
esac
