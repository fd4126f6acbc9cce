# round 6, call c: padding-free units, sym default at P = 8: sym/parity/multirank tests, lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_sym.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_fullsize.py > gpurun_out/r6c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6c_pytest.log; fault_guard gpurun_out/r6c_pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r6c_pytest.log | head -20; exit $rc; }
R=r6c PARTS="sim" bash tools/evidence_profile.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu --repeats 3 > gpurun_out/r6c_bench.json 2> gpurun_out/r6c_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r6c_bench.json').read().strip().splitlines()[-1]); print('cfg3', d['ms_per_step'], d['repeats']['ms_per_step'], d['diag_ms_per_step'])"
