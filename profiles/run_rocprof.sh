#!/bin/bash
# Collects the rocprofv3 summaries committed under profiles/<tag>/ (run on the GPU box via
# gpurun; outputs go to gpurun_out/prof_<tag>/, which gpurun merges back).
#   per config: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
#   (MI355X_MICROARCH.md: TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2 -> one per pass), and a
#   JSON summary (tools/pmc_summary.py) that bench.py reads for roofline.traffic.
# Usage: bash profiles/run_rocprof.sh <round-tag> [configs...]
set -e -o pipefail
TAG=${1:-r01}; shift || true
CONFIGS=${@:-C2 C3 C4 C4-native storage}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
for c in $CONFIGS; do
  mkdir -p $OUT/$c
  case $c in
    *-native) ARGS="--config ${c%-native} --obs native" ;;
    # C5 at one GPU: one batch and no decoded pass (the two-batch run with the decode pass on
    # the comm stream stopped making progress under the kernel trace in round 3)
    C5) ARGS="--config C5 --batches 1 --no-decode --root-rehearsal 0" ;;
    *) ARGS="--config $c" ;;
  esac
  # C4-rezero: every obs row written in full (the flat full-write kernel, bench.py's extra of the name)
  if [ "$c" = C4-rezero ]; then ARGS="--config C4"; export NMMO_OBS_REZERO=1; else unset NMMO_OBS_REZERO; fi
  if [ "$c" = storage ]; then  # experience-storage kernels (tools/bench_storage.py)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c/trace -o run -- \
      python3 tools/bench_storage.py > $OUT/$c/bench_storage.json
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$c/fetch -o run -- \
      python3 tools/bench_storage.py > /dev/null
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$c/write -o run -- \
      python3 tools/bench_storage.py > /dev/null
    python3 tools/pmc_summary.py $OUT/$c > $OUT/$c/pmc.json
    echo "profiled $c"
    continue
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c/trace -o run -- \
    python3 bench.py $ARGS --steps 100 --warmup 20 --no-cpu-baseline --no-extras > $OUT/$c/bench.json
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$c/fetch -o run -- \
    python3 bench.py $ARGS --steps 30 --warmup 5 --no-cpu-baseline --no-extras > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$c/write -o run -- \
    python3 bench.py $ARGS --steps 30 --warmup 5 --no-cpu-baseline --no-extras > /dev/null
  python3 tools/pmc_summary.py $OUT/$c > $OUT/$c/pmc.json
  echo "profiled $c"
done
