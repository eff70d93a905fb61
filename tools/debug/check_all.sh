mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 150 python tools/debug/hang_probe.py --ticks 1500 > gpurun_out/probe.log 2>&1 || { echo PROBE rc=$?; tail -3 gpurun_out/probe.log; exit 1; }
tail -1 gpurun_out/probe.log
timeout -k 10 480 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH rc=$?; tail -5 gpurun_out/bench.err; exit 1; }
echo BENCH OK
