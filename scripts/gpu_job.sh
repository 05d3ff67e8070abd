#!/bin/bash
# One parameterised GPU job (run through gpurun).  Each argument is a step, run in
# order, each under its own time limit; the job stops at the first failing step.
#   test:<pytest args>       e.g. "test:tests/test_netdes.py -k netdes50"
#   bench:<tag>:<bench.py args>
#   prof:<tag>:<bench.py args>          rocprofv3 --kernel-trace --stats
#   trace:<tag>:<bench.py args>         rocprofv3 --kernel-trace --hip-runtime-trace (host gaps)
#   pmc:<tag>:<counters>:<bench.py args> rocprofv3 --pmc (one pass; counters comma-separated)
#   py:<tag>:<script and args>
#   run:<tag>:<program and args>        (a prebuilt binary, e.g. scripts/micro/*)
# Logs: gpurun_out/<tag>.log (tests: gpurun_out/test_<n>.log).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind="${step%%:*}"; rest="${step#*:}"
  case "$kind" in
    test)
      log="gpurun_out/test_${n}.log"
      echo "== step $n: pytest $rest"
      timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $rest > "$log" 2>&1
      rc=$?; tail -4 "$log" ;;
    bench)
      tag="${rest%%:*}"; args="${rest#*:}"; log="gpurun_out/${tag}.log"
      echo "== step $n: bench.py $args"
      timeout -k 10 600 python -u bench.py $args > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    prof)
      tag="${rest%%:*}"; args="${rest#*:}"; log="gpurun_out/${tag}.log"
      echo "== step $n: rocprofv3 --kernel-trace --stats bench.py $args"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${tag}" -o run -- python3 bench.py $args > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    trace)
      tag="${rest%%:*}"; args="${rest#*:}"; log="gpurun_out/${tag}.log"
      echo "== step $n: rocprofv3 --kernel-trace --hip-runtime-trace bench.py $args"
      timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace -d "gpurun_out/${tag}" -o run -- python3 bench.py $args > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    pmc)
      tag="${rest%%:*}"; rest2="${rest#*:}"; ctr="${rest2%%:*}"; args="${rest2#*:}"; log="gpurun_out/${tag}.log"
      echo "== step $n: rocprofv3 --pmc ${ctr//,/ } bench.py $args"
      timeout -s KILL 240 rocprofv3 --pmc ${ctr//,/ } -d "gpurun_out/${tag}" -o run -- python3 bench.py $args > "$log" 2>&1
      rc=$?; tail -2 "$log"
      # the sources this pass measured (scripts/pmc_summary.py records it)
      python3 scripts/src_hash.py > "gpurun_out/${tag}/src_hash.json" ;;
    py)
      tag="${rest%%:*}"; args="${rest#*:}"; log="gpurun_out/${tag}.log"
      echo "== step $n: python $args"
      timeout -k 10 600 python -u $args > "$log" 2>&1
      rc=$?; tail -6 "$log" ;;
    run)
      tag="${rest%%:*}"; args="${rest#*:}"; log="gpurun_out/${tag}.log"
      echo "== step $n: $args"
      timeout -k 10 120 $args > "$log" 2>&1
      rc=$?; tail -6 "$log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then echo "step $n failed (rc=$rc)"; exit $rc; fi
done
