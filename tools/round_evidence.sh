#!/bin/bash
# All GPU evidence of a round in one gpurun call, each step under its own
# time limit (tools/gpu_steps.sh stops at the first fault or timeout):
#   /usr/local/graft/bin/gpurun --timeout 1100 -- 'bash tools/round_evidence.sh'
# then, back in the build container:
#   python3 tools/update_profiles.py rNN c2 c3 c5   (+ copy the row / probe outputs)
bash tools/gpu_steps.sh \
  "pyt|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|100|python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "b1|200|python bench.py --config c1" \
  "b2|200|python bench.py --config c2" \
  "b3|200|python bench.py --config c3" \
  "b4|200|python bench.py --config c4" \
  "b5|200|python bench.py --config c5" \
  "p2|240|bash tools/profile_config.sh c2 gpurun_out/prof_c2" \
  "p3|240|bash tools/profile_config.sh c3 gpurun_out/prof_c3" \
  "p5|240|bash tools/profile_config.sh c5 gpurun_out/prof_c5" \
  "f1|200|python bench.py --config f1" \
  "f3|200|python bench.py --config f3" \
  "f4|200|python bench.py --config f4" \
  "pr|300|bash tools/profile_rows.sh gpurun_out/prof_rows" \
  "v2|200|./tools/rx_variants c2 5" \
  "v3|200|./tools/rx_variants c3 5" \
  "v5|200|./tools/rx_variants c5 3" \
  "sp|100|./tools/store_probe" \
  "pc|100|./tools/pcie_probe" \
  "io|400|python tools/io_path_bench.py 1048576"
