mkdir -p gpurun_out/r03_phases
DIAG_WARMUP=5 PP3_DIAG_OUT=gpurun_out/r03_phases timeout -k 10 200 python tests/diag_phases.py > gpurun_out/r03_phases/phases_w5.txt 2>&1; echo rc=$?
cat gpurun_out/r03_phases/phases_w5.txt | head -24
