cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/p3d gpurun_out/p3r
D3_MODES=delta timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p3d -o run --output-format csv -- python3 tests/bench_suite.py d3 > gpurun_out/p3d.log 2>&1 &&
D3_MODES=reference timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p3r -o run --output-format csv -- python3 tests/bench_suite.py d3 > gpurun_out/p3r.log 2>&1; echo rc=$?
