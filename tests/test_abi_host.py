"""Host-side checks that need no GPU: the C-ABI library loads and exports every entry point
include/unet_hip.h declares, the ctypes mirror of `unet_view` matches the C layout, workspace
queries are consistent, and the Python binding rejects bad arguments before any launch."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "unet_hip.h"


def _declared():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(unet_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from unet_amd import _lib
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    # and the binding declares exactly those
    assert set(_lib.SIGNATURES) == set(names)
    assert lib.unet_abi_version() == _lib.ABI_VERSION


def _prototypes():
    """name -> parameter count of every prototype in the header."""
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for name, params in re.findall(r"\b(unet_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", txt):
        params = params.strip()
        out[name] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_binding_argument_counts_match_header():
    """Every ctypes argtypes list has exactly as many entries as the C prototype has parameters
    (a mismatch only surfaces as a ctypes ArgumentError at the first call on the GPU box)."""
    from unet_amd import _lib
    protos = _prototypes()
    assert set(protos) == set(_lib.SIGNATURES)
    for name, (_, argtypes) in _lib.SIGNATURES.items():
        assert len(argtypes) == protos[name], (name, len(argtypes), protos[name])


def test_view_struct_layout_matches_c():
    from unet_amd._lib import UnetView
    # int32 x4, 6 pointers, float, int32, uint64 -> 16 + 48 + 8 + 8 = 80 bytes, 8-aligned
    assert ctypes.sizeof(UnetView) == 80
    assert UnetView.src0.offset == 16 and UnetView.drop_rate.offset == 64 and UnetView.drop_seed.offset == 72


def test_workspace_queries():
    from unet_amd import _lib
    q = _lib.query
    # ceil(1000/128) tiles x C x float2 (256-B aligned) + one chunk record x C x double2 of finalize
    # scratch (256-B aligned) + ceil(C/64) arrival counters
    assert q("unet_bn_partials_size", 1000, 64) == 8 * 64 * 8 + 1 * 64 * 16 + 4
    assert q("unet_bn_partials_size", 0, 64) == 0
    # BN-backward slabs [S][2C] float | double chunk rows, one per 64 slabs | ceil(C/64) counters
    assert q("unet_bn_stats_partials_size", 300, 64) == 300 * 128 * 4 + 5 * 128 * 8 + 1 * 4
    assert q("unet_bn_stats_partials_size", 1, 8) == 256 + 256 + 1 * 4
    assert q("unet_bn_stats_partials_size", 100, 1024) == 100 * 2048 * 4 + 2 * 2048 * 8 + 16 * 4
    for fn, args in [("unet_dwconv3x3_bwd_filter_workspace", (16, 256, 256, 64)),
                     ("unet_pointwise_bwd_filter_workspace", (16 * 65536, 64, 64)),
                     ("unet_bn_relu_bwd_workspace", (16 * 65536, 64)),
                     ("unet_conv_transpose2x2_bwd_workspace", (16, 128, 128, 128, 64)),
                     ("unet_dice_workspace", (16, 65536, 1)),
                     ("unet_head_bwd_workspace", (16, 256, 256, 64, 1))]:
        b = q(fn, *args)
        assert b > 0 and b % 256 == 0, (fn, b)
        assert q(fn, *([0] + list(args[1:]))) == 0


def test_invalid_arguments_fail_without_gpu():
    """Argument validation happens on the host side of the ABI: no kernel is launched."""
    from unet_amd import _lib
    lib = _lib.load()
    rc = lib.unet_pointwise_fwd(None, 10, 4, 4, None, None, None, None)
    assert rc < 0
    assert b"null pointer" in lib.unet_last_error()
    v = _lib.UnetView()
    v.mode = 7
    rc = lib.unet_dwconv3x3_fwd(ctypes.byref(v), 1, 4, 4, None, None, None)
    assert rc < 0 and b"bad view mode" in lib.unet_last_error()
    rc = lib.unet_meaniou_update(None, None, 10, 2, -1.0, None, None)
    assert rc < 0


def test_ops_refuse_cpu_tensors():
    import torch
    from unet_amd import ops
    x = torch.zeros(1, 4, 4, 8)
    with pytest.raises(ValueError, match="no CPU path"):
        ops.dwconv3x3_fwd(ops.View.plain(x), 1, 4, 4, torch.zeros(72), torch.zeros_like(x))


def test_engine_refuses_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from unet_amd.engine import UNetEngine
    with pytest.raises(RuntimeError, match="no CPU execution path"):
        UNetEngine((32, 32, 3))


from unet_amd import _lib  # noqa: E402


@pytest.fixture(scope="module")
def lib():
    return _lib.load()


# argument validation of every entry point: null pointers and zero sizes are refused (or, for the
# size / support queries, answered with 0) before any device call -- runs without a GPU
_QUERIES = ("_workspace", "_size", "_slabs", "_supported", "unet_abi_version", "unet_last_error",
            "unet_event_destroy", "unet_sepconv_set_schedule")


@pytest.mark.parametrize("name", sorted(_lib.SIGNATURES))
def test_entry_point_rejects_null_arguments(lib, name):
    res, args = _lib.SIGNATURES[name]
    f = getattr(lib, name)
    f.restype, f.argtypes = res, args
    vals = []
    for a in args:
        if a in (ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_uint64):
            vals.append(0)
        elif a is ctypes.c_float:
            vals.append(0.0)
        else:
            vals.append(None)
    r = f(*vals)
    if name.endswith(_QUERIES) or name in _QUERIES:
        return
    assert r != 0, f"{name} accepted null / zero arguments"
    assert lib.unet_last_error(), f"{name} refused without an error message"
