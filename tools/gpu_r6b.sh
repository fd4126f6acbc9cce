# round 6, call b: the world-8 tests, then cfg3 and sim-8 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_multirank.py -k "world8 or symmetric" tests/test_gpu_rccl.py > gpurun_out/r6b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6b_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --repeats 3 > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err && \
timeout -k 10 300 python bench.py --no-cpu --repeats 3 --sim-world 8 > gpurun_out/r6b_sim8.json 2> gpurun_out/r6b_sim8.err && \
SVGD_PHI_SYM=1 timeout -k 10 300 python bench.py --no-cpu --repeats 3 --sim-world 8 > gpurun_out/r6b_sim8_sym.json 2> gpurun_out/r6b_sim8_sym.err
rc=$?; echo "bench rc=$rc"
for f in r6b_bench r6b_sim8 r6b_sim8_sym; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d.get('repeats',{}).get('ms_per_step'), d['per_rank'][0].get('diag_ms_per_step'), d['per_rank'][0]['host_ms_per_step']['threads'])" || true; done
exit $rc
