set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5final; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python bench.py > $O/bench.json 2> $O/bench.err || exit 13
PMC_FILTER=predict_vec scripts/pmc.sh $O/pmc -- python scripts/encode_probe.py 4 > $O/pmc.log 2>&1 || exit 14
echo FINAL OK
