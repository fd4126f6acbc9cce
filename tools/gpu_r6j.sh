# round 6, call j: event-free step end (seq in pinned memory) + finish restricted
# to the touched run: the affected GPU tests, then cfg3 / sim-8 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6j
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sym.py tests/test_gpu_speculative.py tests/test_gpu_track.py tests/test_gpu_median_paths.py \
  tests/test_gpu_rccl.py tests/test_gpu_multirank.py tests/test_gpu_host_model_step.py \
  > gpurun_out/r6j/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r6j/pytest.log
fault_guard gpurun_out/r6j/pytest.log
[ $rc -eq 0 ] || exit $rc
for f in cfg3 sim8; do
  a=""; [ $f = sim8 ] && a="--sim-world 8"
  timeout -k 10 300 python bench.py --no-cpu --repeats 5 $a > gpurun_out/r6j/$f.json 2> gpurun_out/r6j/$f.err || exit 1
  fault_guard gpurun_out/r6j/$f.err
  python3 -c "import json; d=json.loads(open('gpurun_out/r6j/$f.json').read().strip().splitlines()[-1]); r=d['per_rank'][0]; print('$f', round(d['ms_per_step'],4), d['repeats']['ms_per_step'], r.get('diag_ms_per_step'), r['phases_ms_per_step'])"
done
