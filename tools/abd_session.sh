mkdir -p gpurun_out/abd
PP3_LIB_PATH=$PWD/ab/base.so timeout -k 10 120 python3 tools/ab_diff.py gpurun_out/abd/base.npz 3 && PP3_LIB_PATH=$PWD/ab/fused.so timeout -k 10 120 python3 tools/ab_diff.py gpurun_out/abd/fused.npz 3
