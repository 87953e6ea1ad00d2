"""Resource budget of the gfx950 kernels in libmtcp_gpu.so (no GPU needed).

The launch (mtcp_gpu.hip grid_for) puts two 256-thread workgroups on every
CU, i.e. two waves per SIMD, so every rx_kernel instantiation must fit in
256 VGPRs + AGPRs; a kernel that grows past that silently runs at half the
waves (measured: the size-sorted C3 schedule at 254 VGPRs + 32 AGPRs took
193 us instead of 135 us).  No kernel may spill to scratch.  The metadata
comes from the code object's AMDGPU notes (llvm-objcopy, clang-offload-bundler,
llvm-readelf from /opt/rocm/llvm).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mtcp_amd", "lib", "libmtcp_gpu.so")
LLVM = "/opt/rocm/llvm/bin"


def _kernels(tmp_path):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(os.path.exists(t) for t in tools) or not os.path.exists(LIB):
        pytest.skip("ROCm LLVM tools or the built library are missing")
    objcopy, bundler, readelf = tools
    fb, co = tmp_path / "fb.bin", tmp_path / "co.o"
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fb}", LIB, str(tmp_path / "lib.tmp")],
                   check=True)
    subprocess.run([bundler, "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"],
                   check=True)
    notes = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    kernels, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*(-\s+)?\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1):                       # a new list item begins
            cur = {}
            kernels.append(cur)
        if cur is not None:
            cur[m.group(2)] = m.group(3)
    return [k for k in kernels if "name" in k and "vgpr_count" in k]


def test_no_scratch_and_rx_kernels_fit_two_waves_per_simd(tmp_path):
    ks = _kernels(tmp_path)
    rx = [k for k in ks if "rx_kernel" in k["name"]]
    assert len(rx) >= 12, [k["name"] for k in ks]      # 3 modes x RSS on/off x schedules
    for k in ks:
        assert int(k["private_segment_fixed_size"]) == 0, k
        assert int(k.get("vgpr_spill_count", 0)) == 0, k
    for k in rx:
        regs = int(k["vgpr_count"]) + int(k.get("agpr_count", 0))
        assert regs <= 256, f"{k['name']}: {regs} VGPR+AGPR > 256 (two waves per SIMD)"
