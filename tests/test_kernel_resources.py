"""Register and scratch budget of the product library's gfx950 kernels, read from the code-object
metadata embedded in libunet_hip.so (host only: no GPU).  A kernel that spills to scratch memory
pays a global-memory round trip per spilled value.  Only LDS-A-tile fused-forward variants that
the default step does not launch (dropout views of the 64-column tile, max-pool views) spill
today; the register-A kernels the step runs must stay within their registers."""
import os
import re
import shutil
import struct
import subprocess
import tempfile
from pathlib import Path

import pytest

LIB = Path(__file__).resolve().parents[1] / "unet-image-segmentation_amd" / "unet_amd" / "libunet_hip.so"
LLVM = Path("/opt/rocm/lib/llvm/bin")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tool(name):
    p = LLVM / name
    return str(p) if p.exists() else shutil.which(name)


def _kernel_resources():
    """{kernel symbol: (scratch bytes per lane, spilled VGPRs)} over every gfx950 code object."""
    objcopy, readelf = _tool("llvm-objcopy"), _tool("llvm-readelf")
    if not (LIB.exists() and objcopy and readelf):
        pytest.skip("needs the built libunet_hip.so and llvm-objcopy / llvm-readelf")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        # (an explicit output file: without one objcopy rewrites the library in place, which
        # changes its sha256 -- the key the committed PMC traffic summaries are pinned to)
        subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", str(LIB), os.path.join(d, "lib.so")],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
        pos, k = 0, 0
        while (i := blob.find(BUNDLE_MAGIC, pos)) >= 0:
            (entries,) = struct.unpack_from("<Q", blob, i + 24)
            p = i + 32
            for _ in range(entries):
                off, size, tlen = struct.unpack_from("<QQQ", blob, p)
                triple = blob[p + 24:p + 24 + tlen].decode()
                p += 24 + tlen
                if "gfx950" not in triple or size == 0:
                    continue
                elf = os.path.join(d, f"co{k}.elf")
                k += 1
                open(elf, "wb").write(blob[i + off:i + off + size])
                notes = subprocess.run([readelf, "--notes", elf], check=True, capture_output=True,
                                       text=True).stdout
                name = None
                scratch = spills = 0
                for line in notes.splitlines():
                    m = re.match(r"\s+\.name:\s+(\S+)", line)
                    if m:
                        if name is not None:
                            out[name] = (scratch, spills)
                        name, scratch, spills = m.group(1), 0, 0
                        continue
                    m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
                    if m:
                        scratch = int(m.group(1))
                    m = re.match(r"\s+\.vgpr_spill_count:\s+(\d+)", line)
                    if m:
                        spills = int(m.group(1))
                if name is not None:
                    out[name] = (scratch, spills)
            pos = i + len(BUNDLE_MAGIC)
    assert k > 0, "no gfx950 code object in libunet_hip.so"
    return out


def test_only_lds_a_tile_fused_forward_uses_scratch():
    res = _kernel_resources()
    assert len(res) > 100
    allowed = re.compile(r"sepconv_fwd_kernel")
    offenders = {n: r for n, r in res.items() if r[0] > 0 and not allowed.search(n)}
    assert not offenders, f"kernels spilling to scratch: {offenders}"


def test_register_a_fused_forward_does_not_spill():
    # every register-A fused forward (sepconv_rk_kernel, the one the step runs at >= 64^2), and in
    # particular the split-precision 128-column tile at its three-wave register cap
    res = _kernel_resources()
    tiles = {n: r for n, r in res.items() if "sepconv_rk_kernel" in n}
    assert any(re.search(r"ELi128ELb[01]ELb1E", n) for n in tiles), "no 128-column split-precision kernels"
    assert all(r == (0, 0) for r in tiles.values()), tiles


def test_persistent_fused_forward_keeps_its_staging_in_registers():
    # the persistent split-precision forward (sepconv_px_kernel) holds two register sets of staged
    # loads; a private array in scratch would put vmcnt(0) waits into its k-loop and drain the
    # prefetch (round 4: a [2][3] uint4 array did exactly that)
    res = _kernel_resources()
    px = {n: r for n, r in res.items() if "sepconv_px_kernel" in n}
    assert len(px) >= 48, len(px)
    assert all(r == (0, 0) for r in px.values()), {n: r for n, r in px.items() if r != (0, 0)}
