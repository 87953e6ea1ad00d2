"""Per-launch time of the dispatched rx kernel on small and large batches
(HIP events on the launch stream); python tools/small_batch_probe.py"""
import sys, json, numpy as np, torch
sys.path.insert(0, "/root/repo")
from mtcp_amd import gpu, pktgen
dev = torch.device("cuda", 0)
# a non-null stream: the kernels and the events share it (a null handle
# would send the launches to the context's own stream)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
for size, n in [(1500, 4096), (1500, 65536), ("bimodal", 4096), (9000, 4096), (1500, 1 << 20)]:
    desc, nbytes = pktgen.layout(n, size, 6, 7)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    o = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    gpu.pktgen_dev(b, d, n, 6, 7)
    with gpu.Context(0, rss=False) as ctx:
        for _ in range(20): ctx.rx_chunk_dev(b, d, n, 6, o, stream=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 200
        e0.record(st)
        for _ in range(reps): ctx.rx_chunk_dev(b, d, n, 6, o, stream=st)
        e1.record(st); torch.cuda.synchronize()
        print(json.dumps({"size": size, "n": n, "us_per_launch": round(e0.elapsed_time(e1) / reps * 1e3, 2)}))
