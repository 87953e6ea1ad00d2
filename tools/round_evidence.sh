#!/bin/bash
# All GPU evidence of a round in one gpurun call, each step under its own
# time limit (tools/gpu_steps.sh stops at the first fault or timeout):
#   /usr/local/graft/bin/gpurun --timeout 1150 -- 'bash tools/round_evidence.sh'
# then, back in the build container:
#   python3 tools/update_profiles.py rNN c1 c2 c3 c3_compact c5 f1 f3   (+ copy the row / probe outputs)
# Order: the PMC passes first, then `update_profiles.py --traffic` writes
# profiles/traffic_<cfg>.json for THIS build, then the bench lines, so every
# committed bench line quotes the traffic of the library it measured.
bash tools/gpu_steps.sh \
  "pyt|300|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "smoke|100|python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "p2|200|bash tools/profile_config.sh c2 gpurun_out/prof_c2" \
  "p3|200|bash tools/profile_config.sh c3 gpurun_out/prof_c3" \
  "p3c|200|bash tools/profile_config.sh c3_compact gpurun_out/prof_c3_compact" \
  "p5|240|bash tools/profile_config.sh c5 gpurun_out/prof_c5" \
  "pf1|200|bash tools/profile_config.sh f1 gpurun_out/prof_f1" \
  "p1|200|bash tools/profile_config.sh c1 gpurun_out/prof_c1" \
  "pf3|200|bash tools/profile_config.sh f3 gpurun_out/prof_f3" \
  "tr|60|python3 tools/update_profiles.py --traffic c1 c2 c3 c3_compact c5 f1 f3" \
  "bc1|150|python bench.py --config c1" \
  "bc2|150|python bench.py --config c2" \
  "bc3|150|python bench.py --config c3" \
  "bc3_compact|150|python bench.py --config c3 --record compact" \
  "bc4|150|python bench.py --config c4" \
  "bc5|200|python bench.py --config c5" \
  "bf1|150|python bench.py --config f1" \
  "bf3|150|python bench.py --config f3" \
  "bf4|150|python bench.py --config f4" \
  "c2x5|300|for i in 1 2 3 4 5; do python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; done" \
  "bn8|300|MTCP_BENCH_DEVICE=0 python3 bench.py --gpus 8 --per-gpu 131072 --steps 20 --warmup 5" \
  "txhang|120|MTCP_GPU_TX=1 MTCP_GPU_PIPELINE=1 MTCP_GPU_TX_STALL_AFTER=2 MTCP_GPU_STALL_US=1500000 MTCP_GPU_WAIT_TIMEOUT_MS=100 oracle/_ref/dropin_tx /tmp/txhang.bin 4096 observe" \
  "txsw|120|MTCP_GPU_TX=0 oracle/_ref/dropin_tx /tmp/txsw.bin 4096 observe && MTCP_GPU_TX=1 oracle/_ref/dropin_tx /tmp/txgpu.bin 4096 observe && cmp /tmp/txhang.bin /tmp/txsw.bin && cmp /tmp/txgpu.bin /tmp/txsw.bin && echo tx-frames-identical" \
  "dmap|400|OUT=gpurun_out/dispatch_map.jsonl bash tools/dispatch_map.sh" \
  "pr|240|bash tools/profile_rows.sh gpurun_out/prof_rows" \
  "xctx|120|python -u tools/cross_ctx_probe.py > gpurun_out/cross_ctx.json" \
  "free|120|python -u tools/free_sync_probe.py > gpurun_out/free_sync.jsonl" \
  "stop|120|MTCP_GPU_PIPELINE=1 MTCP_GPU_TX=0 MTCP_GPU_WAIT_TIMEOUT_MS=100 MTCP_GPU_STALL_AFTER=1 MTCP_GPU_STALL_US=1500000 oracle/_ref/dropin_rx tests/golden/rx_buf.bin tests/golden/rx_desc.bin /tmp/stop.bin observe stop > gpurun_out/shutdown_inflight.json" \
  "wp|120|./tools/wave_probe 1500 64 1024 4096 16384 32768 && ./tools/wave_probe 9000 64 4096 16384 && ./tools/wave_probe 64 64 4096 16384 65536"
