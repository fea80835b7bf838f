"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every
symbol ``include/recsys_hip.h`` declares (no compute calls: no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "recsys_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t) (rs_\w+)\(", text, flags=re.M)))


def test_header_declares_the_hot_path():
    syms = declared_symbols()
    for required in ["rs_gemm", "rs_attn_fwd", "rs_attn_bwd", "rs_embed_fwd", "rs_embed_bwd",
                     "rs_layernorm_fwd", "rs_layernorm_bwd", "rs_sampled_logits_fwd", "rs_bce_fwd",
                     "rs_ce_fwd", "rs_adam_step"]:
        assert required in syms


def test_library_exports_every_declared_symbol():
    import rbm_amd._lib as L
    assert os.path.exists(L.LIB_PATH), "build the library first (__graft_entry__.build())"
    h = ctypes.CDLL(L.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(h, s), s
    assert set(L.SIGNATURES) == set(declared_symbols())
    assert L.lib().rs_abi_version() == 1


def test_grouped_wgrad_slab_size_host_function():
    """rs_wgrad_grouped_slab_numel is host-only: the Python sizing helper must agree with it."""
    import rbm_amd._lib as L
    from rbm_amd import ops
    shapes = [(128, 128), (256, 128), (64, 64)]
    arr = (L.WgradProblem * 3)(*[L.WgradProblem(None, N, None, K, N, K, None, None) for N, K in shapes])
    for M, rows in [(25600, 640), (111, 64), (64, 128)]:
        assert L.lib().rs_wgrad_grouped_slab_numel(3, arr, M, rows) == ops.wgrad_grouped_slab_numel(shapes, M, rows)


def test_product_path_does_not_import_oracle():
    pkg = os.path.join(ROOT, "recommender-baseline-model_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f
