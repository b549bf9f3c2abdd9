cd $GRAFT_REPO_ROOT
LDSP_DEBUG_PLL=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | cut -c1-300
