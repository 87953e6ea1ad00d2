#!/usr/bin/env python3
"""Rehearse bench.py's N>1 path on a one-GPU box: every rank uses device 0.

torch.distributed.run sets LOCAL_RANK = 0..N-1; this wrapper maps all ranks
onto the box's single GPU (the ranks then share it, so the timings mean
nothing) and runs bench.py's main() unchanged, to exercise the gloo
rendezvous, the sharding, the barriers and the max-over-ranks reduction on
real HIP devices before the driver's 8-GPU run.
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29531 tools/bench_shared_gpu.py --gpus 2 ...
"""
import os
import sys

os.environ["LOCAL_RANK"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

bench.main()
