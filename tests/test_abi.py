"""C-ABI surface checks that need no GPU: the library loads, exports every
symbol include/algodsp.h declares, and fails loudly (no CPU fallback) when
no device is present."""
import ctypes as C
import pathlib
import subprocess

import numpy as np
import pytest

from algodsp import _lib, conv


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    syms = _lib.exported_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T " in line}
    assert set(syms) <= exported


def test_header_declares_every_exported_symbol():
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T " in line and line.split()[-1].startswith("ad_")}
    assert exported <= set(_lib.exported_symbols())


def test_version_and_last_error():
    L = _lib.lib()
    assert L.ad_version() >= 1
    assert isinstance(L.ad_last_error(), bytes)


def _no_gpu():
    return _lib.device_count() == 0


@pytest.mark.skipif(not _no_gpu(), reason="a GPU is visible; covered by the gpu tests")
def test_no_cpu_fallback_without_device():
    with pytest.raises(_lib.ADError) as e:
        conv.NewStreamingOverlapSave([1.0, 0.5], 4)
    assert e.value.code == _lib.AD_ERR_NO_DEVICE
    with pytest.raises(_lib.ADError) as e:
        conv.Direct([1.0, 2.0], [1.0])
    assert e.value.code == _lib.AD_ERR_NO_DEVICE


def test_validation_errors_precede_device_use():
    """Reference sentinel errors are reported before any device work."""
    with pytest.raises(conv.ErrEmptyKernel):
        conv.NewStreamingOverlapSave([], 4)
    with pytest.raises(conv.ErrInvalidArgument):
        conv.NewStreamingOverlapSave([1.0], 0)
    with pytest.raises(conv.ErrEmptyKernel):
        conv.NewOverlapSave([], 0)
    with pytest.raises(conv.ErrInvalidBlockSize):
        conv.NewOverlapSave(np.ones(10), 300)
    with pytest.raises(conv.ErrEmptyImpulseResponse):
        conv.NewPartitionedConvolution([], 7, 13)
    with pytest.raises(conv.ErrInvalidBlockOrder):
        conv.NewPartitionedConvolution([1.0], 0, 13)
    with pytest.raises(conv.ErrInvalidBlockOrder):
        conv.NewPartitionedConvolution([1.0], 8, 7)
    with pytest.raises(conv.ErrEmptyInput):
        conv.Direct([], [1.0])
    with pytest.raises(conv.ErrEmptyKernel):
        conv.Direct([1.0], [])


def test_bench_world_size_mismatch_exits_before_gpu():
    """bench.py --gpus N refuses a launcher world size that disagrees with N
    (before anything touches the GPU) instead of silently running fewer ranks."""
    import os
    import subprocess
    import sys

    root = pathlib.Path(__file__).resolve().parent.parent
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_comm_rejects_bad_arguments_without_gpu():
    """ad_comm_create / ad_mixdown_reduce validate before touching RCCL."""
    import ctypes as C

    L = _lib.lib()
    h = C.c_void_p()
    uid = (C.c_uint8 * 128)()
    assert L.ad_comm_create(uid, 2, 5, 0, C.byref(h)) == _lib.AD_ERR_INVALID_ARGUMENT
    assert not h.value
    assert L.ad_mixdown_reduce(None, None, 2, 10, 10, 0, None, 10, 0, None) == _lib.AD_ERR_INVALID_ARGUMENT


def test_eq_noise_estimate_host_only():
    """ad_fx_eq_noise (the engine-choice estimate of ad_fx_chain_set_eq) runs
    on the host: config 5's EQ at 48 kHz estimates 3.6e-13 (under the
    time-parallel engine's 4.5e-13 gate); an unstable section gives +inf,
    including ADVICE r4's a1 = 4, a2 = 2 (pole at -3.41), for which the old
    test d = (1 - a2)((1 + a2)^2 - a1^2) > 0 still held."""
    from algodsp import design

    L = _lib.lib()

    def noise(secs):
        tab = np.ascontiguousarray(np.asarray(secs, dtype=np.float64))
        out = C.c_double()
        _lib.check(L.ad_fx_eq_noise(tab.ctypes.data_as(C.POINTER(C.c_double)), tab.shape[0], 1, C.byref(out)))
        return out.value

    from algodsp.processors import section_table

    eq = design.config5_eq(48000.0)
    tab = np.concatenate([section_table(co, g) for co, g in eq])
    assert 3.0e-13 < noise(tab) < 4.5e-13
    unstable = tab.copy()
    unstable[0, 4:6] = [4.0, 2.0]
    assert noise(unstable) == float("inf")
    edge = tab.copy()
    edge[1, 5] = 1.0
    assert noise(edge) == float("inf")
    with pytest.raises(_lib.ErrInvalidArgument):
        bad = C.c_double()
        _lib.check(L.ad_fx_eq_noise(None, 2, 1, C.byref(bad)))


# Each value a reference setter rejects (compressor.go:16-23; core.go:10-12,
# 131-198, 542-564), applied to NewCompressor's defaults at 48 kHz.
BAD_COMPRESSOR_VALUES = [
    ("ratio", 100.5), ("ratio", 0.5), ("ratio", float("nan")),
    ("knee_db", 24.5), ("knee_db", -0.1),
    ("attack_ms", 0.05), ("attack_ms", 1000.5),
    ("release_ms", 0.5), ("release_ms", 5001.0),
    ("rms_window_ms", 0.5), ("rms_window_ms", 1001.0),
    ("threshold_db", float("nan")), ("threshold_db", float("inf")),
    ("makeup_db", float("nan")), ("makeup_db", float("-inf")),
    ("sidechain_low_cut_hz", 0.5), ("sidechain_high_cut_hz", 0.5),
    ("sidechain_low_cut_hz", 24000.0), ("sidechain_high_cut_hz", 30000.0),
    ("sidechain_low_cut_hz", -1.0), ("sidechain_high_cut_hz", float("nan")),
    ("sample_rate", 0.0), ("topology", 2), ("detector_mode", -1),
]
GOOD_COMPRESSOR_EDGES = [
    ("ratio", 1.0), ("ratio", 100.0), ("knee_db", 0.0), ("knee_db", 24.0),
    ("attack_ms", 0.1), ("attack_ms", 1000.0), ("release_ms", 1.0), ("release_ms", 5000.0),
    ("rms_window_ms", 1.0), ("rms_window_ms", 1000.0),
    ("sidechain_low_cut_hz", 1.0), ("sidechain_high_cut_hz", 23999.0),
]


def _comp_cfg(**kv):
    cfg = _lib.CompressorConfig()
    _lib.lib().ad_compressor_default_config(C.byref(cfg), 48000.0)
    for k, v in kv.items():
        setattr(cfg, k, v)
    return cfg


@pytest.mark.parametrize("field,value", BAD_COMPRESSOR_VALUES)
def test_compressor_validation_rejects_setter_ranges(field, value):
    rc = _lib.lib().ad_compressor_validate(C.byref(_comp_cfg(**{field: value})))
    assert rc == _lib.AD_ERR_INVALID_ARGUMENT, (field, value)


def test_compressor_validation_low_must_be_below_high():
    L = _lib.lib()
    assert L.ad_compressor_validate(C.byref(_comp_cfg(sidechain_low_cut_hz=6000.0, sidechain_high_cut_hz=6000.0))) \
        == _lib.AD_ERR_INVALID_ARGUMENT
    assert L.ad_compressor_validate(C.byref(_comp_cfg(sidechain_low_cut_hz=7000.0, sidechain_high_cut_hz=80.0))) \
        == _lib.AD_ERR_INVALID_ARGUMENT
    assert L.ad_compressor_validate(C.byref(_comp_cfg(sidechain_low_cut_hz=80.0, sidechain_high_cut_hz=6000.0))) \
        == _lib.AD_OK
    assert L.ad_compressor_validate(None) == _lib.AD_ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("field,value", GOOD_COMPRESSOR_EDGES)
def test_compressor_validation_accepts_range_edges(field, value):
    assert _lib.lib().ad_compressor_validate(C.byref(_comp_cfg(**{field: value}))) == _lib.AD_OK


def test_integration_snippets_name_real_abi():
    """Every C.ad_* function and C.AD_* constant INTEGRATION.md's Go snippets
    call exists in include/algodsp.h, and every Go snippet that registers with
    the reference names the reference line it matches."""
    import re

    root = pathlib.Path(__file__).resolve().parents[1]
    doc = (root / "INTEGRATION.md").read_text()
    header = (root / "include" / "algodsp.h").read_text()
    funcs = set(re.findall(r"\bC\.(ad_[a-z0-9_]+)\(", doc))
    consts = set(re.findall(r"\bC\.(AD_[A-Z0-9_]+)\b", doc))
    types = set(re.findall(r"\bC\.(ad_[a-z0-9_]+)\b", doc)) - funcs
    assert funcs and consts
    missing = [f for f in funcs if not re.search(r"\b" + f + r"\s*\(", header)]
    missing += [c for c in consts if not re.search(r"#define\s+" + c + r"\b", header)]
    missing += [t for t in types if not re.search(r"\b" + t + r"\b", header)]
    assert not missing, missing
    # the registrations carry the reference's own types and line numbers
    for needle in ("registry.OpEntry{", "ProcessBlock: processBlock", "registry.go:17",
                   "func(ctx effectchain.Context) (effectchain.Runtime, error)", "registry.go:24",
                   "conv.RegisterBackend", "convolution.go:35"):
        assert needle in doc, needle
