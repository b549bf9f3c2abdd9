cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "
import sys, json, torch; sys.argv=['bench.py']
import bench, liquiddsp as L
print(json.dumps(bench.host_path(L, torch.device('cuda', 0))))
" > gpurun_out/hp.log 2>&1 || { tail -5 gpurun_out/hp.log; exit 1; }
tail -1 gpurun_out/hp.log
