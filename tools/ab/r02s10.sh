# final tree: full GPU test suite
set -o pipefail
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; exit $rc
