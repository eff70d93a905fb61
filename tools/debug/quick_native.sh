# native/wire obs change check: GPU tests, then C4-native and C5 bench lines (no extras)
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputest.log; exit 1; }
tail -1 gpurun_out/gputest.log
for rep in 1 2; do
timeout -k 10 150 python bench.py --config C4 --obs native --no-cpu-baseline --no-extras > gpurun_out/c4n_$rep.json 2> gpurun_out/c4n_$rep.err || { echo C4N rc=$?; tail -5 gpurun_out/c4n_$rep.err; exit 1; }
timeout -k 10 150 python bench.py --config C5 --no-cpu-baseline --no-extras > gpurun_out/c5_$rep.json 2> gpurun_out/c5_$rep.err || { echo C5 rc=$?; tail -5 gpurun_out/c5_$rep.err; exit 1; }
done
echo OK
