#!/bin/bash
# round 6: GPU visibility as bench.visible_gpus sees it, the -m gpu suite, the d3 trace, bench.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
python -c "
import sys,os; sys.path.insert(0,'.'); import bench
print('visible_gpus', bench.visible_gpus(), 'kfd', bench.kfd_fds())
t='/sys/class/kfd/kfd/topology/nodes'
for n in sorted(os.listdir(t)):
    p=open(os.path.join(t,n,'properties')).read().split()
    d=dict(zip(p[::2],p[1::2])); print(n, d.get('simd_count'), d.get('drm_render_minor'))
print(sorted(os.listdir('/dev/dri')))
" > gpurun_out/r06_visible.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r06_gpu_tests.log 2>&1 || exit $?
bash scripts/gpu_steps.sh profd3 bench
