mkdir -p gpurun_out/cs
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_regressors.py -k "small_batch_tiles or batch_invariance or hier" -x -q --timeout 120 --timeout-method thread > gpurun_out/cs/t.log 2>&1 || exit 1
for B in 1 8 16; do MP_CONV_SMALL=0 timeout -k 10 120 python tools/time_pose.py --batch $B --profile || exit 1; timeout -k 10 120 python tools/time_pose.py --batch $B --profile || exit 1; done > gpurun_out/cs/time.log 2>&1 || exit 1
for v in 0 1 0 1; do MP_GRAPH_CONV_DENSE=$v timeout -k 10 200 python tools/time_regressors.py 256 || exit 1; done > gpurun_out/cs/reg.log 2>&1 || exit 1
MP_GRAPH_CONV_DENSE=0 timeout -k 10 200 python tools/profile_graph.py hier 256 > gpurun_out/cs/prof_hier0.log 2>&1 || exit 1
MP_GRAPH_CONV_DENSE=1 timeout -k 10 200 python tools/profile_graph.py hier 256 > gpurun_out/cs/prof_hier1.log 2>&1 || exit 1
