export PP3_REPORT_DIR=gpurun_out
rm -f gpurun_out/gpu_reports.jsonl
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo tests_rc=$?; tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --gather --no-extras --no-cpu-baseline --no-latency-floor > gpurun_out/bench_gather1.json 2>&1; echo gather_rc=$?; tail -c 800 gpurun_out/bench_gather1.json
timeout -k 10 200 python tools/step_trace.py --steps 300 > gpurun_out/step_trace.jsonl 2>&1; echo trace_rc=$?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 -d gpurun_out/pcs -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras > gpurun_out/pcs.log 2>&1; echo pcs_rc=$?; tail -5 gpurun_out/pcs.log; ls -R gpurun_out/pcs | head
