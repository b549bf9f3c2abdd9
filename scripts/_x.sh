cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --cpu-seconds 2 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
python -c "
import json; r=json.loads([l for l in open('gpurun_out/b.log') if l.startswith('{')][-1])
print(r['value'], r['config']); print(r['components']['resampler_64Mi']); print(r['cpu_baseline'])"
