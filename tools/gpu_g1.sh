# round-6 session: ADVICE fixes, RCCL fallback, one-pass select, placement probe, per-shape C4 ledger
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/g5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_fused_passes_gpu.py tests/test_exact_gpu.py "tests/test_distributed_gpu.py::test_world2_ops_on_shards" "tests/test_distributed_gpu.py::test_world2_ops_on_shards_p2p" tests/test_bench.py tests/test_mpi_bridge_gpu.py tests/test_ops_gpu.py tests/test_fullsize_gpu.py > $O/tests.log 2>&1
timeout -k 10 300 python -u tools/placement_probe.py --out $O/placement.json > $O/placement.log 2>&1
SSP_LEDGER_DETAIL=1 SSP_LEDGER_TIMING=dispatch timeout -k 10 200 python -u tools/solver_ledger.py --configs C4-shard --out $O/c4_detail.json > $O/c4_detail.log 2>&1
