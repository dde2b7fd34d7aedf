set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r06e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06e_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06e_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r06e_smoke.log; exit 1; }
tail -1 gpurun_out/r06e_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06e_bench.json 2> gpurun_out/r06e_bench.err || { echo BENCH FAILED; tail gpurun_out/r06e_bench.err; exit 1; }
cut -c1-300 gpurun_out/r06e_bench.json
