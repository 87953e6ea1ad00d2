#!/bin/bash
# The round-end sequence as the driver runs it (GPU tests, smoke, default
# bench), plus repeats of the headline line for its spread on one box.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/final_check.sh'
bash tools/gpu_steps.sh \
  "fc_pyt|300|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "fc_smoke|100|python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "fc_bench|150|python bench.py" \
  "fc_rep|300|for i in 1 2 3 4 5; do python bench.py --cpu-baseline off --pcie off --small-batch off; done"
