"""Host-side DenseNet plan (no GPU): layer geometry and parameter layout from
the C ABI agree with the oracle's reading of densenet.py:135-196."""
import ctypes

import numpy as np
import pytest

from oracle import densenet as od


def _plan(arch, n=4, batch=16):
    from mpi_opt_amd import _lib

    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.mpo_dn_create(ctypes.byref(arch.c_struct()), n, batch, ctypes.byref(h))
    return L, rc, h


@pytest.mark.parametrize("img,depth,blocks,growth,nbf", [((32, 32, 3), 10, 3, 12, 16), ((9, 11, 2), 7, 2, 5, 7),
                                                        ((150, 94, 5), 10, 3, 12, 16)])
def test_plan_geometry_matches_oracle(img, depth, blocks, growth, nbf):
    from mpi_opt_amd import _lib
    from mpi_opt_amd.densenet import KIND_NAMES, DenseNetArch, param_shapes

    arch = DenseNetArch(img_dim=img, nb_classes=3, depth=depth, nb_dense_block=blocks, growth_rate=growth,
                        nb_filter=nbf)
    L, rc, h = _plan(arch)
    assert rc == 0, L.mpo_last_error()
    try:
        sz = _lib.MpoDnSizes()
        assert L.mpo_dn_sizes(h, ctypes.byref(sz)) == 0
        ref = od.arch_layers(img_dim=img, nb_classes=3, depth=depth, nb_dense_block=blocks, growth_rate=growth,
                             nb_filter=nbf)
        assert sz.n_layers == len(ref)
        geom = (ctypes.c_int32 * 8)()
        offs = (ctypes.c_int64 * 6)()
        layers = []
        spans = []
        for i, r in enumerate(ref):
            assert L.mpo_dn_layer(h, i, geom, offs) == 0
            g = list(geom)
            ly = dict(kind=KIND_NAMES[g[0]], stage=g[1], H=g[2], W=g[3], cin=g[4], cout=g[5], ks=g[6], coff=g[7])
            layers.append(ly)
            for k in ("kind", "H", "W", "cin", "cout"):
                assert ly[k] == r[k], (i, k)
            if r["kind"] in ("dense", "trans"):
                assert ly["ks"] == r["ks"] and ly["coff"] == r["coff"]
            o = list(offs)
            if ly["kind"] == "conv0":
                spans.append((o[0], 9 * ly["cin"] * ly["cout"]))
            else:
                spans += [(o[1], ly["H"]), (o[2], ly["H"])]
                if ly["kind"] == "head":
                    spans += [(o[0], ly["cin"] * ly["cout"]), (o[5], ly["cout"])]
                else:
                    spans.append((o[0], ly["ks"] ** 2 * ly["cin"] * ly["cout"]))
        # parameter tensors are disjoint and inside the per-member block
        spans.sort()
        for (a0, n0), (a1, _) in zip(spans, spans[1:]):
            assert a0 + n0 <= a1
        assert spans[-1][0] + spans[-1][1] <= sz.n_params
        P, _ = param_shapes(layers)
        Po, _ = od.param_shapes(ref)
        assert P == Po
        assert sz.act_floats > 0
    finally:
        L.mpo_dn_destroy(h)


def test_plan_rejects_bad_depth_and_wide_images():
    from mpi_opt_amd.densenet import DenseNetArch

    L, rc, h = _plan(DenseNetArch(depth=11))
    assert rc == 1 and b"3 N + 4" in L.mpo_last_error()
    L, rc, h = _plan(DenseNetArch(img_dim=(8, 300, 3)))
    assert rc == 3


def test_flops_reference_config():
    from mpi_opt_amd.densenet import flops_per_sample_fwd, flops_per_sample_train

    layers = od.arch_layers()
    assert flops_per_sample_fwd(layers) == od.flops_per_sample_fwd(layers)
    assert flops_per_sample_train(layers) == od.flops_per_sample_train(layers)
    assert np.isclose(flops_per_sample_fwd(layers) / 1e6, 22.8, atol=0.5)


def test_python_layer_geometry_matches_oracle_and_spec_ingestion():
    from mpi_opt_amd.densenet import DenseNetArch
    from mpi_opt_amd.models import DenseNetModel, DenseNetSpec, spec_from_json, test_densenet

    for img, depth, blocks in [((32, 32, 3), 10, 3), ((9, 11, 2), 7, 2), ((150, 94, 5), 13, 3)]:
        arch = DenseNetArch(img_dim=img, nb_classes=4, depth=depth, nb_dense_block=blocks)
        ref = od.arch_layers(img_dim=img, nb_classes=4, depth=depth, nb_dense_block=blocks)
        got = arch.layers()
        assert [{k: l[k] for k in ("kind", "H", "W", "cin", "cout")} for l in got] == \
               [{k: l[k] for k in ("kind", "H", "W", "cin", "cout")} for l in ref]
    # the lr dimension (10**-2 here) is compiled into the Keras model and lost by to_json
    # (base_model.py:67-73): the trainer's lr applies
    spec = spec_from_json(DenseNetModel(input_shape=(32, 32, 3)).build([10, 3, 12, 0.0, 16, -2]), lr=1e-3)
    assert isinstance(spec, DenseNetSpec) and spec.lr == 1e-3
    assert spec.arch.key() == ((32, 32, 3), 3, 10, 3, 12, 16)
    assert spec.flops_per_sample_train() == od.flops_per_sample_train(od.arch_layers(img_dim=(32, 32, 3),
                                                                                     nb_classes=3))
    with pytest.raises(ValueError):
        spec_from_json(test_densenet(dropout_rate=0.2))


def test_hbm_models_follow_the_pooled_transition_epilogue(monkeypatch):
    """The transition's AvgPool2 runs in the 1x1 conv's epilogue when the streamed
    1x1 kernel applies (even H, W % 8 == 0; r05) or the staged conv's row chunk is
    even (csrc/densenet.hip enqueue_forward): the reference grid's transitions
    (32x32, 16x16) have no separate pool pass and no pre-pool tensor in either HBM
    model, and their 1x1 convs are dn_conv1x1_kernel's; an 18-wide image (7-row
    chunks, 18 % 8 != 0) keeps both."""
    from mpi_opt_amd import densenet as dn

    ref = dn.DenseNetArch().layers()
    by = dn.hbm_bytes_train_by_kernel(ref, 100, 0)
    assert "dn_pool_fwd_kernel" not in by and by["dn_pool_bwd_kernel"] > 0 and by["dn_conv1x1_kernel"] > 0
    odd = dn.DenseNetArch(img_dim=(18, 18, 3)).layers()
    assert dn.hbm_bytes_train_by_kernel(odd, 100, 0)["dn_pool_fwd_kernel"] > 0
    fused_floor, fused_by = dn.hbm_bytes_train(ref, 100, 0), sum(by.values())
    monkeypatch.setattr(dn, "_pool_fused", lambda H, W: False)
    monkeypatch.setattr(dn, "_conv1x1_streamed", lambda ly: False)
    # unfused, each transition writes its pre-pool output and the pool pass reads it back
    saved = 4 * 100 * sum(2 * ly["H"] * ly["W"] * ly["cout"] for ly in ref if ly["kind"] == "trans")
    assert dn.hbm_bytes_train(ref, 100, 0) - fused_floor == saved
    assert sum(dn.hbm_bytes_train_by_kernel(ref, 100, 0).values()) - fused_by == saved
