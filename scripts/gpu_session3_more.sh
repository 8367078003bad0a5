# end-of-round refresh of the other BASELINE rows on the final tree: 70B TP=1, batch 1, HTTP path
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/s3b
timeout -k 10 900 python bench.py --model llama-3-70b --batch 64 --steps 2 --json-out gpurun_out/s3b/rag_70b.json > gpurun_out/s3b/rag_70b.log 2>&1 || { tail -5 gpurun_out/s3b/rag_70b.log; exit 1; }
cut -c1-200 gpurun_out/s3b/rag_70b.json
timeout -k 10 400 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/s3b/rag_b1.json > gpurun_out/s3b/rag_b1.log 2>&1 || { tail -5 gpurun_out/s3b/rag_b1.log; exit 2; }
cut -c1-200 gpurun_out/s3b/rag_b1.json
timeout -k 10 900 python -u bench.py --via-http --json-out gpurun_out/s3b/http_bench.json > gpurun_out/s3b/http_bench.log 2>&1 || { tail -20 gpurun_out/s3b/http_bench.log; exit 3; }
grep '"metric"' gpurun_out/s3b/http_bench.log | cut -c1-400
