set -e
timeout -k 10 200 python3 tools/group_proto.py 20 5 > gpurun_out/gp/a.log 2>&1; cat gpurun_out/gp/a.log
timeout -k 10 200 python3 tools/group_proto.py 200 200 1,4,8 > gpurun_out/gp/b.log 2>&1; cat gpurun_out/gp/b.log
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 tools/group_proto.py 20 5 4,8 > gpurun_out/gp/c.log 2>&1; cat gpurun_out/gp/c.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python3 tools/group_proto.py 20 5 8,16 > gpurun_out/gp/d.log 2>&1; cat gpurun_out/gp/d.log
