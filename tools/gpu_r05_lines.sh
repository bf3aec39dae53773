#!/bin/bash
# Round-5 session: job timing, ingest tests + ingest A/B, shuffled line, 2-rank gloo C3 rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_jobs.py::test_aggregate_job_on_device_row_batches > gpurun_out/r05_job.txt 2>&1 || { echo job failed; exit 1; }
ZKAGG_LIB=$PWD/zipkin_amd/libzkagg_snappy2.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_ingest.py tests/test_gpu_reference_vectors.py > gpurun_out/r05_ingest_tests.txt 2>&1 || { echo ingest tests failed; tail -30 gpurun_out/r05_ingest_tests.txt; exit 1; }
AB_ROUNDS=3 timeout -k 10 600 bash tools/ing_ab.sh cur snappy2 > gpurun_out/r05_ab_ingest.txt 2>&1 || { echo ing ab failed; cat gpurun_out/r05_ab_ingest.txt; exit 1; }
timeout -k 10 400 python -u bench.py --workload ingest --steps 10 > gpurun_out/r05_ingest.json 2> gpurun_out/r05_ingest.err || { echo ingest bench failed; exit 1; }
timeout -k 10 400 python -u bench.py --order shuffled --steps 10 > gpurun_out/r05_shuffled.json 2> gpurun_out/r05_shuffled.err || { echo shuffled failed; tail gpurun_out/r05_shuffled.err; exit 1; }
ZK_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload c3 --records 200000000 --steps 5 --warmup 2 > gpurun_out/r05_gloo2_c3.json 2> gpurun_out/r05_gloo2_c3.err || { echo gloo failed; tail gpurun_out/r05_gloo2_c3.err; exit 1; }
echo session done
