#!/bin/bash
# A/B of the group kernels' aligned phase-2 form (rx_group_kernel AL 1 vs 0),
# then the round-end check.
bash tools/gpu_steps.sh \
  "al_pyt|300|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "al_wp|200|for r in 1 2 3; do WP_ONLY=empty,g4,g4noal,g16,g16noal ./tools/wave_probe 64 4096 16384 65536 && WP_ONLY=empty,g4,g4noal,g16,g16noal ./tools/wave_probe 1500 4096 16384 32768; done" \
  "al_c1|200|for r in 1 2 3; do python bench.py --config c1 --cpu-baseline off --pcie off --small-batch off; done"
