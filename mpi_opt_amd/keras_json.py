"""Keras functional-model JSON for DenseNet, without Keras.

The reference's DenseNet builders hand the trainer ``Model.to_json()`` of the
functional model ``densenet.DenseNet`` builds (/root/reference/densenet.py:
135-196; reached from mpiLAPI.py:197-201 ``test_densenet`` and
base_model.py:62-73 ``DenseNetModel.build``).  The trainer rebuilds the network
from that JSON (mpi_learn ``ModelFromJsonTF``).  Keras is absent here and on
the GPU box, so this module does both sides:

* :func:`densenet_json` records the same layer graph densenet.py builds --
  initial 3x3 conv, per dense layer BN(axis=1) -> ELU -> 3x3 conv(growth) ->
  concat of *all* the block's features (``merge(list_feat, mode='concat',
  concat_axis=-1)``), per transition BN -> ELU -> 1x1 conv -> AvgPool2, then
  BN -> ELU -> GAP -> Dense softmax, l2(weight_decay) on every conv / BN / Dense
  -- and serialises it as Keras 2.0/2.1 writes a functional ``Model``: a
  ``layers`` list of ``{name, class_name, config, inbound_nodes}``,
  ``input_layers`` / ``output_layers``, auto-generated layer names.  (Keras
  2.0-2.1 is what densenet.py needs: its Keras-1 keywords go through Keras 2's
  legacy interface and ``merge(mode='concat')`` is the legacy ``Merge`` layer,
  removed in Keras 2.2.)
* :func:`densenet_arch_from_json` ingests such a JSON -- ``Merge`` (mode
  concat) or Keras >= 2.2 ``Concatenate``; Keras 2 or Keras 1 field names
  (``filters``/``nb_filter``, ``padding``/``border_mode``, ``use_bias``/``bias``)
  -- into a :class:`~mpi_opt_amd.densenet.DenseNetArch`.  It infers the
  architecture's parameters, rebuilds the canonical graph from them and
  requires the two graphs to be identical up to layer names (canonical
  post-order walk from the output), so any topology the DenseNet population
  engine does not implement is rejected with the first differing layer named.

Compile-time arguments (``Adam(lr)`` in base_model.py:67-71 / mpiLAPI.py:199)
are not part of ``to_json()``; as in the reference the trainer's optimizer lr
applies (a dead dimension, like topclass's ``llr``).
"""
from __future__ import annotations

import json

import numpy as np

KERAS_VERSION = "2.1.6"


def _l2(wd):
    # Keras holds regularizer factors as floatx (float32) and serialises that value
    return {"class_name": "L1L2", "config": {"l1": 0.0, "l2": float(np.float32(wd))}}


def _init(name, **cfg):
    return {"class_name": name, "config": cfg}


HE_UNIFORM = _init("VarianceScaling", scale=2.0, mode="fan_in", distribution="uniform", seed=None)
GLOROT_UNIFORM = _init("VarianceScaling", scale=1.0, mode="fan_avg", distribution="uniform", seed=None)


class _Graph:
    """Records layers in creation order with Keras's auto-naming."""

    def __init__(self):
        self.layers = []
        self.counts = {}

    def add(self, class_name, base, config, inputs, name=None):
        if name is None:
            self.counts[base] = self.counts.get(base, 0) + 1
            name = f"{base}_{self.counts[base]}"
        cfg = {"name": name, "trainable": True, **config}
        nodes = [[[i, 0, 0, {}] for i in inputs]] if inputs else []
        self.layers.append({"name": name, "class_name": class_name, "config": cfg, "inbound_nodes": nodes})
        return name


def _bn(g, x, wd):
    return g.add("BatchNormalization", "batch_normalization", {
        "axis": 1, "momentum": 0.99, "epsilon": 0.001, "center": True, "scale": True,
        "beta_initializer": _init("Zeros"), "gamma_initializer": _init("Ones"),
        "moving_mean_initializer": _init("Zeros"), "moving_variance_initializer": _init("Ones"),
        "beta_regularizer": _l2(wd), "gamma_regularizer": _l2(wd), "beta_constraint": None,
        "gamma_constraint": None}, [x])


def _conv(g, x, filters, ks, wd, name=None):
    return g.add("Conv2D", "conv2d", {
        "filters": int(filters), "kernel_size": [ks, ks], "strides": [1, 1], "padding": "same",
        "data_format": "channels_last", "dilation_rate": [1, 1], "activation": "linear", "use_bias": False,
        "kernel_initializer": HE_UNIFORM, "bias_initializer": _init("Zeros"), "kernel_regularizer": _l2(wd),
        "bias_regularizer": None, "activity_regularizer": None, "kernel_constraint": None,
        "bias_constraint": None}, [x], name=name)


def _elu(g, x):
    return g.add("Activation", "activation", {"activation": "elu"}, [x])


def _dropout(g, x, rate):
    return g.add("Dropout", "dropout", {"rate": float(rate), "noise_shape": None, "seed": None}, [x])


def densenet_json(nb_classes, img_dim, depth, nb_dense_block, growth_rate, nb_filter, dropout_rate=None,
                  weight_decay=1e-4, name="DenseNet"):
    """``DenseNet(...).to_json()`` (densenet.py:135-196) as Keras 2.1 writes it."""
    assert (depth - 4) % 3 == 0, "Depth must be 3 N + 4"
    nb_layers = (depth - 4) // 3
    wd = weight_decay
    g = _Graph()
    inp = g.add("InputLayer", "input", {"batch_input_shape": [None, *[int(v) for v in img_dim]],
                                        "dtype": "float32", "sparse": False}, [])
    x = _conv(g, inp, nb_filter, 3, wd, name="initial_conv2D")

    def denseblock(x, f):
        feats = [x]
        for _ in range(nb_layers):
            c = _conv(g, _elu(g, _bn(g, x, wd)), growth_rate, 3, wd)
            if dropout_rate:
                c = _dropout(g, c, dropout_rate)
            feats.append(c)
            x = g.add("Merge", "merge", {"mode": "concat", "mode_type": "raw", "concat_axis": -1, "dot_axes": -1,
                                         "output_shape": None, "output_shape_type": "raw", "output_mask": None,
                                         "output_mask_type": "raw", "arguments": {}}, list(feats))
            f += growth_rate
        return x, f

    f = nb_filter
    for _ in range(nb_dense_block - 1):
        x, f = denseblock(x, f)
        x = _conv(g, _elu(g, _bn(g, x, wd)), f, 1, wd)
        if dropout_rate:
            x = _dropout(g, x, dropout_rate)
        x = g.add("AveragePooling2D", "average_pooling2d", {"pool_size": [2, 2], "padding": "valid",
                                                            "strides": [2, 2], "data_format": "channels_last"}, [x])
    x, f = denseblock(x, f)
    x = _elu(g, _bn(g, x, wd))
    x = g.add("GlobalAveragePooling2D", "global_average_pooling2d", {"data_format": "channels_last"}, [x])
    out = g.add("Dense", "dense", {
        "units": int(nb_classes), "activation": "softmax", "use_bias": True, "kernel_initializer": GLOROT_UNIFORM,
        "bias_initializer": _init("Zeros"), "kernel_regularizer": _l2(wd), "bias_regularizer": _l2(wd),
        "activity_regularizer": None, "kernel_constraint": None, "bias_constraint": None}, [x])
    return json.dumps({"class_name": "Model",
                       "config": {"name": name, "layers": g.layers, "input_layers": [[inp, 0, 0]],
                                  "output_layers": [[out, 0, 0]]},
                       "keras_version": KERAS_VERSION, "backend": "tensorflow"})


# --------------------------------------------------------------------------
# ingestion
# --------------------------------------------------------------------------
def _get(cfg, *keys, default=None):
    for k in keys:
        if k in cfg:
            return cfg[k]
    return default


def _reg_l2(r):
    if r is None:
        return None
    c = r.get("config", r)
    return float(c.get("l2", 0.0))


def _signature(cls, cfg):
    """What the population engine depends on in one layer (Keras 1 and 2 field names)."""
    if cls == "InputLayer":
        return ("input", tuple(cfg["batch_input_shape"][1:]))
    if cls in ("Conv2D", "Convolution2D"):
        ks = _get(cfg, "kernel_size")
        ks = tuple(ks) if ks is not None else (cfg["nb_row"], cfg["nb_col"])
        return ("conv", int(_get(cfg, "filters", "nb_filter")), ks, tuple(_get(cfg, "strides", "subsample",
                                                                            default=(1, 1))),
                _get(cfg, "padding", "border_mode"), bool(_get(cfg, "use_bias", "bias", default=True)),
                _get(cfg, "activation", default="linear"), _reg_l2(_get(cfg, "kernel_regularizer", "W_regularizer")))
    if cls == "BatchNormalization":
        return ("bn", int(cfg.get("axis", -1)), float(cfg.get("epsilon", 1e-3)), float(cfg.get("momentum", 0.99)),
                bool(cfg.get("center", True)), bool(cfg.get("scale", True)),
                _reg_l2(cfg.get("gamma_regularizer")), _reg_l2(cfg.get("beta_regularizer")))
    if cls == "Activation":
        return ("act", cfg["activation"])
    if cls == "Merge":
        if cfg.get("mode") != "concat":
            return ("merge", cfg.get("mode"))
        return ("concat", int(cfg.get("concat_axis", -1)) % 4)
    if cls == "Concatenate":
        return ("concat", int(cfg.get("axis", -1)) % 4)
    if cls == "AveragePooling2D":
        return ("avgpool", tuple(cfg["pool_size"]), tuple(cfg.get("strides") or cfg["pool_size"]),
                _get(cfg, "padding", "border_mode", default="valid"))
    if cls == "GlobalAveragePooling2D":
        return ("gap",)
    if cls == "Dense":
        return ("dense", int(_get(cfg, "units", "output_dim")), cfg.get("activation"),
                bool(_get(cfg, "use_bias", "bias", default=True)),
                _reg_l2(_get(cfg, "kernel_regularizer", "W_regularizer")),
                _reg_l2(_get(cfg, "bias_regularizer", "b_regularizer")))
    if cls == "Dropout":
        return ("dropout", float(_get(cfg, "rate", "p")))
    return ("unsupported", cls)


def _layers_of(doc):
    if doc.get("class_name") not in ("Model", "Functional"):
        raise ValueError(f"not a functional Keras model: class_name {doc.get('class_name')!r}")
    cfg = doc["config"]
    layers = {l["name"]: l for l in cfg["layers"]}
    outs = cfg.get("output_layers") or []
    if len(outs) != 1 or len(cfg.get("input_layers") or []) != 1:
        raise ValueError("DenseNet JSON must have one input and one output layer")
    return layers, outs[0][0]


def _inputs(layer):
    nodes = layer.get("inbound_nodes") or []
    if len(nodes) > 1:
        raise ValueError(f"layer {layer['name']} is applied more than once (shared layers are not supported)")
    return [n[0] for n in nodes[0]] if nodes else []


def _canonical(layers, out):
    """Post-order walk from the output: [(signature, [canonical input ids])]."""
    ids, seq, names = {}, [], []

    def visit(name):
        if name in ids:
            return ids[name]
        if name not in layers:
            raise ValueError(f"inbound layer {name!r} is not defined")
        l = layers[name]
        ins = [visit(i) for i in _inputs(l)]
        ids[name] = len(seq)
        seq.append((_signature(l["class_name"], l["config"]), ins))
        names.append(name)
        return ids[name]

    import sys

    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, 10 * len(layers) + 100))
    try:
        visit(out)
    finally:
        sys.setrecursionlimit(old)
    return seq, names


def densenet_arch_from_json(json_str):
    """A functional DenseNet JSON -> (DenseNetArch, weight_decay).  Raises
    ValueError naming the first layer that differs from densenet.py's graph."""
    from .densenet import DenseNetArch

    doc = json.loads(json_str) if isinstance(json_str, str) else json_str
    layers, out = _layers_of(doc)
    seq, names = _canonical(layers, out)
    sigs = [s for s, _ in seq]
    inp = [s for s in sigs if s[0] == "input"]
    convs = [s for s in sigs if s[0] == "conv"]
    dense = [s for s in sigs if s[0] == "dense"]
    if len(inp) != 1 or not convs or len(dense) != 1:
        raise ValueError("not a DenseNet graph (needs one input, convolutions and one Dense head)")
    img_dim = tuple(int(v) for v in inp[0][1])
    if len(img_dim) != 3:
        raise ValueError(f"input shape {img_dim}: expected (rows, cols, channels)")
    nb_filter = convs[0][1]
    threes = [s for s in convs[1:] if s[2] == (3, 3)]
    growth = threes[0][1] if threes else 0
    nb_dense_block = sum(1 for s in sigs if s[0] == "avgpool") + 1
    if not threes or len(threes) % nb_dense_block:
        raise ValueError("dense layers are not split evenly over the dense blocks")
    nb_layers = len(threes) // nb_dense_block
    wd = convs[0][7] if convs[0][7] is not None else 0.0
    drops = {s[1] for s in sigs if s[0] == "dropout"}
    dropout_rate = drops.pop() if len(drops) == 1 else (None if not drops else -1.0)
    if dropout_rate == -1.0:
        raise ValueError("dropout layers with different rates")
    ref = json.loads(densenet_json(dense[0][1], img_dim, 3 * nb_layers + 4, nb_dense_block, growth, nb_filter,
                                   dropout_rate=dropout_rate, weight_decay=wd))
    rlayers, rout = _layers_of(ref)
    rseq, _ = _canonical(rlayers, rout)
    for i, ((s, ins), (rs, rins)) in enumerate(zip(seq, rseq)):
        if s != rs or ins != rins:
            raise ValueError(f"layer {names[i]!r}: {s} with inputs {ins} differs from densenet.py's graph "
                             f"({rs} with inputs {rins})")
    if len(seq) != len(rseq):
        raise ValueError(f"{len(seq)} layers reach the output, densenet.py's graph has {len(rseq)}")
    if dropout_rate:
        raise ValueError("DenseNet population trains dropout_rate 0 (the reference grid, base_model.py:88)")
    arch = DenseNetArch(img_dim=img_dim, nb_classes=int(dense[0][1]), depth=3 * nb_layers + 4,
                        nb_dense_block=nb_dense_block, growth_rate=int(growth), nb_filter=int(nb_filter))
    return arch, wd
