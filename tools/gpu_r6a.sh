# round 6, call a: multi-rank tests (true host reduce-scatter, world-8),
# symmetric-pass tests (fused row-stream hand-over), rccl; cfg3 and sim-8 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_sym.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py > gpurun_out/r6a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6a_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --repeats 3 > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err && \
timeout -k 10 300 python bench.py --no-cpu --repeats 3 --sim-world 8 > gpurun_out/r6a_sim8.json 2> gpurun_out/r6a_sim8.err && \
SVGD_PHI_SYM=1 timeout -k 10 300 python bench.py --no-cpu --repeats 3 --sim-world 8 > gpurun_out/r6a_sim8_sym.json 2> gpurun_out/r6a_sim8_sym.err
rc=$?; echo "bench rc=$rc"
for f in r6a_bench r6a_sim8 r6a_sim8_sym; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d.get('repeats',{}).get('ms_per_step'), d['per_rank'][0].get('diag_ms_per_step'), d['per_rank'][0]['host_ms_per_step']['threads'])" || true; done
exit $rc
