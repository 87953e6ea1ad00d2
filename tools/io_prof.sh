#!/bin/bash
# GPU timeline of the io_module path (tests/c/rxloop over gpu_module.c), one
# thread, pipelined and synchronous, 64 B and 1500 B frames:
#   /usr/local/graft/bin/gpurun -- 'bash tools/io_prof.sh'
# -> gpurun_out/prof_io_<size>_p<0|1>/*.db (rocprofv3 SQLite: kernel
# dispatches, memory copies, HIP API calls)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for size in 64 1500; do
  timeout -k 10 120 python tools/io_path_bench.py 262144 --dump /tmp/io$size $size
  for p in 0 1; do
    MTCP_GPU_PIPELINE=$p timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace \
      -d gpurun_out/prof_io_${size}_p$p -o io -- ./tests/c/rxloop /tmp/io$size/chunk.bin \
      /tmp/io$size/desc.bin /tmp/io$size/out.bin timing 1 > gpurun_out/prof_io_${size}_p$p.log 2>&1
  done
done
