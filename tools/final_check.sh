#!/bin/bash
# The round-end sequence as the driver runs it (GPU tests, smoke, default
# bench), plus repeats of the headline line for its spread on one box.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/final_check.sh'
bash tools/gpu_steps.sh \
  "fc_pyt|300|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "fc_smoke|100|python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "fc_bench|150|python bench.py" \
  "fc_rep|300|for i in 1 2 3 4 5; do python bench.py --cpu-baseline off --pcie off --small-batch off; done" || exit $?
# the self-launched multi-rank path, rehearsed with every rank on device 0
# (the driver's 2/4/8-GPU runs use one device per rank)
bash tools/gpu_steps.sh \
  "fc_n4|200|MTCP_BENCH_DEVICE=0 python bench.py --gpus 4 --per-gpu 262144 --pcie off --small-batch off"
