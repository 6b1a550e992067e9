"""CPU-side checks of the C-ABI library (no compute calls): it loads, exports every entry point
declared in include/mmt.h, and its parameter layout reproduces the reference state_dict key set,
shapes and init kinds (mmt_create needs no device: device tables are created lazily)."""
import ctypes
import os
import re

import pytest
import torch

import mmt_lib as ML
from golden_io import MODEL_FIXTURES, model_fixture

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(REPO, "include", "mmt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mmt_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = ML.lib()
    names = _header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(ML.EXPORTED)
    assert b"gfx950" in L.mmt_version()


def _ctx(meta):
    cfg = ML.MmtConfig()
    cfg.num_modalities = len(meta["V"])
    cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.block_size = meta["n_embd"], meta["n_head"], meta["n_layer"], meta["block_size"]
    for i, v in enumerate(meta["V"]):
        cfg.vocab_sizes[i] = v
        cfg.cross_attention[i] = int(meta["cross"][i])
    ctx = ML.lib().mmt_create(ctypes.byref(cfg))
    assert ctx, ML.lib().mmt_create_error()
    return ctypes.c_void_p(ctx)


@pytest.mark.parametrize("name", MODEL_FIXTURES)
def test_layout_matches_reference_state_dict(name):
    z, meta, cfg, sd, idx, tgt = model_fixture(name)
    L = ML.lib()
    ctx = _ctx(meta)
    try:
        n = L.mmt_param_count(ctx)
        act = L.mmt_param_active_count(ctx)
        buf = ctypes.create_string_buffer(256)
        off, nd, shape, kind = ML.c_i64(), ML.c_i32(), (ML.c_i64 * 2)(), ML.c_i32()
        seen = {}
        covered = torch.zeros(n, dtype=torch.int32)
        for i in range(L.mmt_tensor_count(ctx)):
            assert L.mmt_tensor_info(ctx, i, buf, 256, ctypes.byref(off), ctypes.byref(nd), shape, ctypes.byref(kind)) == 0
            shp = [shape[d] for d in range(nd.value)]
            k = buf.value.decode()
            seen[k] = shp
            numel = 1
            for s in shp:
                numel *= s
            covered[off.value:off.value + numel] += 1
            # layer-norm weights init to one, everything else per Linear/Embedding rules
            if k.endswith("bias"):
                assert kind.value in (1, 3)
            if "ln" in k.split(".")[-2] or "norm" in k:
                assert kind.value in (2, 3), k
            # gradient-free parameters (CrossAttention without KV modalities) sit past the active prefix
            assert (off.value >= act) == (k in meta["grad_none"]), k
        ref = {k: v for k, v in meta["state_dict_shapes"].items() if not k.endswith("tril")}
        assert seen == ref
        assert int(covered.max()) == 1  # no two tensors overlap
    finally:
        L.mmt_destroy(ctx)


def test_create_rejects_unsupported_head_size():
    L = ML.lib()
    cfg = ML.MmtConfig()
    cfg.num_modalities, cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.block_size = 1, 36, 4, 1, 8
    cfg.vocab_sizes[0] = 5
    assert not L.mmt_create(ctypes.byref(cfg))
    assert b"head size" in L.mmt_create_error()


def test_backward_stage_ranges_tile_the_active_prefix():
    z, meta, cfg, sd, idx, tgt = model_fixture("f_small")
    L = ML.lib()
    ctx = _ctx(meta)
    try:
        ranges = []
        b, e = ML.c_i64(), ML.c_i64()
        for s in range(L.mmt_backward_stage_count(ctx)):
            assert L.mmt_backward_stage_range(ctx, s, ctypes.byref(b), ctypes.byref(e)) == 0
            ranges.append((b.value, e.value))
        ranges.sort()
        assert ranges[0][0] == 0
        for (b0, e0), (b1, e1) in zip(ranges, ranges[1:]):
            assert e0 == b1
        assert ranges[-1][1] == L.mmt_param_active_count(ctx)
    finally:
        L.mmt_destroy(ctx)
