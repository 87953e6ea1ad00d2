#!/bin/bash
# All GPU evidence of a round in one gpurun call, each step under its own
# time limit (tools/gpu_steps.sh stops at the first fault or timeout):
#   /usr/local/graft/bin/gpurun --timeout 1150 -- 'bash tools/round_evidence.sh'
# then, back in the build container:
#   python3 tools/update_profiles.py rNN c2 c3 c5   (+ copy the row / probe outputs)
bash tools/gpu_steps.sh \
  "pyt|300|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "smoke|100|python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "b1|150|python bench.py --config c1" \
  "b2|150|python bench.py --config c2" \
  "b3|150|python bench.py --config c3" \
  "b4|150|python bench.py --config c4" \
  "b5|200|python bench.py --config c5" \
  "p2|200|bash tools/profile_config.sh c2 gpurun_out/prof_c2" \
  "p3|200|bash tools/profile_config.sh c3 gpurun_out/prof_c3" \
  "p5|240|bash tools/profile_config.sh c5 gpurun_out/prof_c5" \
  "f1|150|python bench.py --config f1" \
  "f3|150|python bench.py --config f3" \
  "f4|150|python bench.py --config f4" \
  "pr|240|bash tools/profile_rows.sh gpurun_out/prof_rows" \
  "wp|120|./tools/wave_probe 1500 64 1024 4096 16384 32768 && ./tools/wave_probe 9000 64 4096 16384 && ./tools/wave_probe 64 64 4096 16384 65536"
