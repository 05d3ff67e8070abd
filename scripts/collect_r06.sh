#!/bin/bash
# Copy the round-6 evidence judged from gpurun_out/ (scratch) into profiles/:
# PMC summaries (scripts/pmc_summary.py over the timed window's launches, with
# the source_sha256 of the sources measured), rocprofv3 kernel statistics of the
# final traces, the default bench line and its detail record.
set -e
G=gpurun_out
P=profiles
S="python3 scripts/pmc_summary.py"
$S phx_lane_warm_fzr2 --last 49 $G/r06_pmc_c3_fetch $G/r06_pmc_c3_write > $P/r06_pmc_farmer100k_phx_lane_warm_fzr2.json
$S phx_lane_warm_fzr2 --last 49 $G/r06_pmc_c3_sq > $P/r06_pmcsq_farmer100k_phx_lane_warm_fzr2.json
$S phx_lane_warm_fz1 --last 19 $G/r06_pmc_s8_fetch $G/r06_pmc_s8_write > $P/r06_pmc_farmer12k5_phx_lane_warm_fz1.json
$S phx_lane_warm_fz1 --last 19 $G/r06_pmc_s8_sq > $P/r06_pmcsq_farmer12k5_phx_lane_warm_fz1.json
$S phx_lane_warm_fzr2 --last 19 $G/r06_pmc_1m_fetch $G/r06_pmc_1m_write > $P/r06_pmc_farmer1m_phx_lane_warm_fzr2.json
$S phx_lane_all_pk --last 10 $G/r06_pmc_c4_fetch $G/r06_pmc_c4_write > $P/r06_pmc_aircond1k_phx_lane_all_pk.json
$S k_wg_warm --last 10 --skip-idle $G/r06_pmc_c2_fetch $G/r06_pmc_c2_write > $P/r06_pmc_farmercm10_1k_k_wg_warm.json
$S k_wg_warm --last 10 --skip-idle $G/r06_pmc_c5a_fetch $G/r06_pmc_c5a_write > $P/r06_pmc_sslp10k_k_wg_warm.json
$S k_sp_solve --last 10 --skip-idle $G/r06_pmc_c5b_fetch $G/r06_pmc_c5b_write > $P/r06_pmc_netdes10k_k_sp_solve.json
for t in prof c3s8_prof 1m_prof c2_prof c4_prof c5a_prof c5b_prof; do
  cp $G/r06_final_$t/run_kernel_stats.csv $P/r06_final_${t%_prof}_kernel_stats.csv
done
mv $P/r06_final_prof_kernel_stats.csv $P/r06_final_headline_kernel_stats.csv 2>/dev/null || true
cp $G/r06_final_default.log $P/r06_final_bench_default.log
cp $G/r06_final_default_detail.json $P/r06_final_bench_default_detail.json
cp $G/test_1.log $P/r06_final_pytest_gpu_all.log 2>/dev/null || true
cp $G/r06_final_smoke.log $P/r06_final_smoke.log 2>/dev/null || true
