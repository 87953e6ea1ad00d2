#!/bin/bash
# All GPU evidence of a round, in two gpurun calls, each step under its own
# time limit (tools/gpu_steps.sh stops at the first fault or timeout):
#   /usr/local/graft/bin/gpurun --timeout 1150 -- 'bash tools/round_evidence.sh 1'
#   /usr/local/graft/bin/gpurun --timeout 1150 -- 'bash tools/round_evidence.sh 2'
# then, back in the build container:
#   python3 tools/update_profiles.py rNN c1 c2 c3 c3_compact c5 f1 f3   (+ copy the probe outputs)
# Part 1: the GPU suite and smoke, the PMC passes, then `update_profiles.py
# --traffic` writes profiles/traffic_<cfg>.json for THIS build, then the
# bench lines, so every committed bench line quotes the traffic of the
# library it measured.  Part 2: the driver's forms and the io_module probes.
if [ "$1" = 1 ]; then
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
  "bf4|150|python bench.py --config f4"
else
bash tools/gpu_steps.sh \
  "c2x5|300|for i in 1 2 3 4 5; do python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; done" \
  "bn8|300|MTCP_BENCH_DEVICE=0 python3 bench.py --gpus 8 --per-gpu 131072 --steps 20 --warmup 5" \
  "iso|60|python -u -m tests.hwq_isolation" \
  "txhang|120|MTCP_GPU_TX=1 MTCP_GPU_PIPELINE=1 MTCP_GPU_TX_STALL_AFTER=2 MTCP_GPU_STALL_US=1500000 MTCP_GPU_WAIT_TIMEOUT_MS=100 oracle/_ref/dropin_tx /tmp/txhang.bin 4096 observe" \
  "txsw|120|MTCP_GPU_TX=0 oracle/_ref/dropin_tx /tmp/txsw.bin 4096 observe && MTCP_GPU_TX=1 oracle/_ref/dropin_tx /tmp/txgpu.bin 4096 observe && cmp /tmp/txhang.bin /tmp/txsw.bin && cmp /tmp/txgpu.bin /tmp/txsw.bin && echo tx-frames-identical" \
  "xctx|120|python -u tools/cross_ctx_probe.py" \
  "stop|120|MTCP_GPU_PIPELINE=1 MTCP_GPU_TX=0 MTCP_GPU_WAIT_TIMEOUT_MS=100 MTCP_GPU_STALL_AFTER=1 MTCP_GPU_STALL_US=1500000 oracle/_ref/dropin_rx tests/golden/rx_buf.bin tests/golden/rx_desc.bin /tmp/stop.bin observe stop" \
  "adm|600|ADM_THREADS=1,2,4,8,16 python -u tools/admission_probe.py 4"
fi
