#!/bin/bash
# The one GPU-box launcher (run under gpurun from the repo root): named steps, each under its own time limit,
# outputs under gpurun_out/<tag>/; stops at the first failing step (no GPU work after a fault, abort or timeout).
#
#   bash tools/gpu/run.sh <tag> <step> [<step> ...]
#
# steps:
#   smoke                     __graft_entry__.smoke()
#   tests[=f1,f2,...]         pytest -m gpu over tests/ (or the listed test files / node ids)
#   stepab=N:V1,V2[:arch[:lib]]  tools/step_ab.py: graph-replayed step time of option variants ("base", "k=v+k=v"),
#                             optionally of another build (ab_libs/libitsd_hip_<lib>.so)
#   census=N[:arch]           tools/census.py per-launch census of one forward (arch a / c; c: N is the guided batch)
#   timeline=N:op,op,...      tools/timeline.py p5 launch timelines (stamps build ab_libs/libitsd_hip_stamps.so)
#   pmc=N                     PMC passes over one census forward + per-dispatch table + traffic files
#   bench                     python bench.py (the driver's line, all extras)
#   prof                      rocprofv3 --kernel-trace --stats of the bench command (no extras)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
fail() { echo "FAIL $1 (rc=$2)"; [ -n "$3" ] && tail -20 "$3"; exit 1; }
for step in "$@"; do
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  echo "== $step" >&2
  case $name in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || fail smoke $? "$out/smoke.txt"
      tail -2 "$out/smoke.txt" ;;
    tests)
      sel=${arg:-tests}; sel=${sel//,/ }
      log="$out/gpu_tests_$(echo "$arg" | tr -c 'A-Za-z0-9' '_' | cut -c1-40).log"
      timeout -k 10 1100 python -u -m pytest $sel -m gpu -x -v -s --timeout 500 --timeout-method thread > "$log" 2>&1 || fail tests $? "$log"
      tail -1 "$log" ;;
    stepab)
      IFS=: read -r n variants arch lib <<< "$arg"
      f="$out/stepab_${arch:-a}$n${lib:+_$lib}.txt"
      timeout -k 10 400 python tools/step_ab.py --n "$n" --variants "$variants" --arch "${arch:-a}" \
        ${lib:+--lib ab_libs/libitsd_hip_$lib.so} > "$f" 2>&1 || fail stepab $? "$f"
      tail -4 "$f" ;;
    census)
      IFS=: read -r n arch <<< "$arg"
      timeout -k 10 200 python tools/census.py --n "$n" --arch "${arch:-a}" > "$out/census_${arch:-a}$n.txt" 2>&1 || fail census $? "$out/census_${arch:-a}$n.txt" ;;
    timeline)
      IFS=: read -r n ops <<< "$arg"
      timeout -k 10 300 python tools/timeline.py ab_libs/libitsd_hip_stamps.so --n "$n" ${ops//,/ } > "$out/timeline_n$n.txt" 2>&1 || fail timeline $? "$out/timeline_n$n.txt" ;;
    pmc)
      timeout -k 10 900 bash tools/pmc_passes.sh "$out/pmc" --n "${arg:-256}" > "$out/pmc.log" 2>&1 || fail pmc $? "$out/pmc.log"
      python tools/pmc_dispatch.py "$out/pmc" > "$out/pmc_dispatch_table.txt" || echo dispatch_table_fail ;;
    bench)
      timeout -k 10 900 python bench.py > "$out/bench.json" 2> "$out/bench.err" || fail bench $? "$out/bench.err"
      tail -c 400 "$out/bench.json" ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
        timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o bench -- \
          python3 bench.py --no-extras --no-cpu-baseline --no-live-traffic > "$out/prof_bench.json" 2> "$out/prof.err" ) || fail prof $? "$out/prof.err"
      find "$out/prof" -name "*kernel_trace.csv" -delete
      find "$out/prof" -name "*stats.csv" ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "run.sh $tag: all steps done"
