set -e
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_compact.py tests/test_dropin.py tests/test_io_module.py tests/test_gpu_rxq.py > gpurun_out/r3_compact.log 2>&1
for r in 1 2 3; do
timeout -k 10 120 python bench.py --config c3 --steps 200 --warmup 20 --cpu-baseline off --pcie off --small-batch off >> gpurun_out/r3_c3_ab.jsonl
timeout -k 10 120 python bench.py --config c3 --record compact --steps 200 --warmup 20 --cpu-baseline off --pcie off --small-batch off >> gpurun_out/r3_c3_ab.jsonl
done
timeout -k 10 400 bash tools/small_batch_trace.sh gpurun_out/sbt_graph graph
WP_ONLY=empty,empty16,full,nl2,w8nl2,w16nl2,phase1,p1nl2 timeout -k 10 120 ./tools/wave_probe 1500 1024 4096 8192 > gpurun_out/r3_wave_wpb.jsonl
WP_ONLY=empty,empty16,full,nl2,w8nl2,w16nl2 timeout -k 10 120 ./tools/wave_probe 64 1024 2048 4096 >> gpurun_out/r3_wave_wpb.jsonl
