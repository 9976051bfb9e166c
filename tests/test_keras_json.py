"""Keras functional-model JSON ingestion for DenseNet.

The fixture ``tests/golden/densenet_keras_functional.json`` is the graph the
reference's own ``densenet.DenseNet(...)`` (/root/reference/densenet.py:135-196)
builds -- recorded by ``make_keras_densenet_fixture.py`` from a run of that
function against a recording stand-in for the Keras 2.1 layer API -- at BASELINE
configs[4] (CIFAR-10 shape, the base_model.py:84-92 grid architecture)."""
import copy
import json
import os
import random

import pytest

from tests.conftest import GOLDEN

FIXTURE = os.path.join(GOLDEN, "densenet_keras_functional.json")


def _doc():
    with open(FIXTURE) as f:
        return json.load(f)


def test_reference_graph_ingests_to_the_config5_arch():
    from mpi_opt_amd.densenet import DenseNetArch
    from mpi_opt_amd.keras_json import densenet_arch_from_json
    from mpi_opt_amd.models import DenseNetSpec, spec_from_json

    arch, wd = densenet_arch_from_json(_doc())
    assert arch == DenseNetArch(img_dim=(32, 32, 3), nb_classes=10, depth=10, nb_dense_block=3, growth_rate=12,
                                nb_filter=16)
    assert abs(wd - 1e-4) < 1e-10                       # float32-rounded l2(1E-4)
    spec = spec_from_json(json.dumps(_doc()), lr=3e-4)
    assert isinstance(spec, DenseNetSpec) and spec.arch == arch and spec.lr == 3e-4   # to_json drops Adam(lr)


def test_emitter_reproduces_the_reference_graph():
    from mpi_opt_amd.keras_json import _canonical, _layers_of, densenet_json

    ours = json.loads(densenet_json(10, (32, 32, 3), 10, 3, 12, 16))
    a, _ = _canonical(*_layers_of(ours))
    b, _ = _canonical(*_layers_of(_doc()))
    assert a == b
    # and the same auto-generated layer names, in the same creation order
    assert [l["name"] for l in ours["config"]["layers"]] == [l["name"] for l in _doc()["config"]["layers"]]


def test_layer_order_and_names_do_not_matter():
    from mpi_opt_amd.keras_json import densenet_arch_from_json

    d = _doc()
    layers = d["config"]["layers"]
    rename = {l["name"]: f"L{i:03d}" for i, l in enumerate(layers)}
    for l in layers:
        l["name"] = l["config"]["name"] = rename[l["name"]]
        for node in l["inbound_nodes"]:
            for inb in node:
                inb[0] = rename[inb[0]]
    d["config"]["input_layers"][0][0] = rename[d["config"]["input_layers"][0][0]]
    d["config"]["output_layers"][0][0] = rename[d["config"]["output_layers"][0][0]]
    random.Random(0).shuffle(layers)
    assert densenet_arch_from_json(d)[0].depth == 10


def test_keras22_concatenate_and_keras1_field_names():
    from mpi_opt_amd.keras_json import densenet_arch_from_json

    d = _doc()
    for l in d["config"]["layers"]:
        c = l["config"]
        if l["class_name"] == "Merge":
            l["class_name"] = "Concatenate"
            l["config"] = {"name": c["name"], "trainable": True, "axis": -1}
        elif l["class_name"] == "Conv2D":
            l["class_name"] = "Convolution2D"
            k = c.pop("kernel_size")
            c.update(nb_filter=c.pop("filters"), nb_row=k[0], nb_col=k[1], border_mode=c.pop("padding"),
                     bias=c.pop("use_bias"), W_regularizer=c.pop("kernel_regularizer"))
    assert densenet_arch_from_json(d)[0].growth_rate == 12


def _mutate(fn):
    d = _doc()
    fn(d["config"]["layers"])
    return d


@pytest.mark.parametrize("what,fn", [
    ("BN over channels", lambda L: [l["config"].update(axis=-1) for l in L if l["class_name"] == "BatchNormalization"]),
    ("relu for elu", lambda L: next(l for l in L if l["class_name"] == "Activation")["config"].update(activation="relu")),
    ("concat misses a feature", lambda L: next(l for l in L if l["name"] == "merge_2")["inbound_nodes"][0].pop(1)),
    ("5x5 growth conv", lambda L: next(l for l in L if l["name"] == "conv2d_2")["config"].update(kernel_size=[5, 5])),
    ("max pooling", lambda L: next(l for l in L if l["class_name"] == "AveragePooling2D").update(
        class_name="MaxPooling2D")),
    ("biased conv", lambda L: next(l for l in L if l["name"] == "conv2d_1")["config"].update(use_bias=True)),
])
def test_graphs_the_engine_does_not_implement_are_rejected(what, fn):
    from mpi_opt_amd.keras_json import densenet_arch_from_json

    with pytest.raises(ValueError):
        densenet_arch_from_json(_mutate(fn))


def test_dropout_and_weight_decay_are_checked():
    from mpi_opt_amd.models import spec_from_json, test_densenet
    from mpi_opt_amd.keras_json import densenet_json

    with pytest.raises(ValueError, match="dropout"):
        spec_from_json(test_densenet(dropout_rate=0.2))
    with pytest.raises(ValueError, match="weight_decay"):
        spec_from_json(densenet_json(10, (32, 32, 3), 10, 3, 12, 16, weight_decay=5e-4))


@pytest.mark.parametrize("img,depth,blocks,growth,f0,classes", [
    ((9, 11, 2), 7, 2, 5, 6, 4), ((150, 94, 5), 13, 3, 12, 16, 3), ((32, 32, 3), 22, 4, 8, 24, 10)])
def test_round_trip_other_geometries(img, depth, blocks, growth, f0, classes):
    from mpi_opt_amd.densenet import DenseNetArch
    from mpi_opt_amd.keras_json import densenet_arch_from_json, densenet_json

    arch, _ = densenet_arch_from_json(densenet_json(classes, img, depth, blocks, growth, f0))
    assert arch == DenseNetArch(img_dim=img, nb_classes=classes, depth=depth, nb_dense_block=blocks,
                                growth_rate=growth, nb_filter=f0)
