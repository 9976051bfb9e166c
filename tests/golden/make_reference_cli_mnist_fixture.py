"""Generate tests/golden/reference_cli_mnist.json by running the reference's own
code in the build container against recording stand-ins for the packages it
imports (keras, h5py, tensorflow, mpi4py, mpi_learn, skopt -- none is installed
here):

* ``make_parser()`` of /root/reference/hyperparameter_search_option3.py:54-96:
  every flag's option strings, dest, default and type, and the defaults of an
  empty command line;
* ``test_mnist(**params)`` of /root/reference/mpiLAPI.py:138-176, through
  ``BuilderFromFunction(mpi.test_mnist, <option3's mnist space>)`` (option3:22-31,
  126-133): the Sequential layer calls it makes (class and arguments, as the
  Keras 2 API receives them) and the model JSON a Keras 2.1 ``to_json()`` would
  write, for the corners of the space and seeded draws.

Run in the build container (needs /root/reference):
    python tests/golden/make_reference_cli_mnist_fixture.py
The reference is only read here, never at test time; the fixture is data.
"""
import argparse
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
OUT = os.path.join(HERE, "reference_cli_mnist.json")

CALLS = []


class _Recorded:
    """A Keras layer stand-in recording its constructor call."""

    cls = None

    def __init__(self, *args, **kwargs):
        self.args, self.kwargs = list(args), dict(kwargs)


def _layer(cls_name):
    return type(cls_name, (_Recorded,), {"cls": cls_name})


Conv2D = _layer("Conv2D")
MaxPooling2D = _layer("MaxPooling2D")
Dense = _layer("Dense")
Dropout = _layer("Dropout")
Activation = _layer("Activation")
Flatten = _layer("Flatten")

_COUNTS = {}


def _name(base):
    _COUNTS[base] = _COUNTS.get(base, 0) + 1
    return f"{base}_{_COUNTS[base]}"


def _pair(v):
    return list(v) if isinstance(v, (tuple, list)) else [v, v]


def _keras21_config(layer):
    """The layer's get_config() as Keras 2.1.6 writes it (what the call implies)."""
    a, k = layer.args, layer.kwargs
    glorot = {"class_name": "VarianceScaling", "config": {"scale": 1.0, "mode": "fan_avg",
                                                          "distribution": "uniform", "seed": None}}
    zeros = {"class_name": "Zeros", "config": {}}
    if layer.cls == "Conv2D":
        cfg = {"name": _name("conv2d"), "trainable": True, "filters": a[0], "kernel_size": _pair(k["kernel_size"]),
               "strides": [1, 1], "padding": k.get("padding", "valid"), "data_format": "channels_last",
               "dilation_rate": [1, 1], "activation": k.get("activation", "linear") or "linear", "use_bias": True,
               "kernel_initializer": glorot, "bias_initializer": zeros, "kernel_regularizer": None,
               "bias_regularizer": None, "activity_regularizer": None, "kernel_constraint": None,
               "bias_constraint": None}
        if "input_shape" in k:
            cfg = {"name": cfg.pop("name"), "trainable": True, "batch_input_shape": [None, *k["input_shape"]],
                   "dtype": "float32", **{kk: vv for kk, vv in cfg.items() if kk != "trainable"}}
        return cfg
    if layer.cls == "Activation":
        return {"name": _name("activation"), "trainable": True, "activation": a[0]}
    if layer.cls == "MaxPooling2D":
        ps = _pair(k["pool_size"])
        return {"name": _name("max_pooling2d"), "trainable": True, "pool_size": ps, "padding": "valid",
                "strides": ps, "data_format": "channels_last"}
    if layer.cls == "Dropout":
        return {"name": _name("dropout"), "trainable": True, "rate": a[0], "noise_shape": None, "seed": None}
    if layer.cls == "Flatten":
        return {"name": _name("flatten"), "trainable": True}
    if layer.cls == "Dense":
        return {"name": _name("dense"), "trainable": True, "units": a[0], "activation": "linear", "use_bias": True,
                "kernel_initializer": glorot, "bias_initializer": zeros, "kernel_regularizer": None,
                "bias_regularizer": None, "activity_regularizer": None, "kernel_constraint": None,
                "bias_constraint": None}
    raise ValueError(layer.cls)


class Sequential:
    def __init__(self):
        self.layers = []

    def add(self, layer):
        self.layers.append(layer)
        CALLS.append({"class": layer.cls, "args": layer.args, "kwargs": {k: (list(v) if isinstance(v, tuple) else v)
                                                                           for k, v in layer.kwargs.items()}})

    def to_json(self):
        _COUNTS.clear()
        cfgs = [{"class_name": l.cls, "config": _keras21_config(l)} for l in self.layers]
        return json.dumps({"class_name": "Sequential", "config": cfgs, "keras_version": "2.1.6",
                           "backend": "tensorflow"})


def _module(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    m.__path__ = []
    sys.modules[name] = m
    if "." in name:
        parent, child = name.rsplit(".", 1)
        if parent in sys.modules:
            setattr(sys.modules[parent], child, m)
    return m


class _Dim:
    def __init__(self, low, high, name=None, **kw):
        self.low, self.high, self.name = low, high, name


def install_stubs():
    sys.path.insert(0, HERE)
    from make_keras_densenet_fixture import install_stub_keras  # the functional-API stand-in (densenet.py)

    install_stub_keras(None)
    keras = sys.modules["keras"]
    sys.modules["keras.models"].Sequential = Sequential
    layers = sys.modules["keras.layers"]
    for c in (Dense, Dropout, Activation, Flatten, Conv2D, MaxPooling2D):
        setattr(layers, c.cls, c)
    _module("keras.optimizers", Adam=lambda **kw: ("Adam", kw))
    keras.backend = sys.modules["keras.backend"]
    _module("h5py")
    _module("tensorflow")
    _module("mpi4py", MPI=types.SimpleNamespace(COMM_WORLD=None))
    _module("mpi_learn")
    _module("mpi_learn.train")
    _module("mpi_learn.train.algo", Algo=object)
    _module("mpi_learn.train.data", H5Data=object)
    _module("mpi_learn.train.model", ModelFromJsonTF=lambda comm, json_str=None: json_str)
    _module("mpi_learn.train.GanModel", GANBuilder=object)
    _module("mpi_learn.utils", import_keras=lambda *a, **k: None)
    _module("mpi_learn.mpi")
    _module("mpi_learn.mpi.manager")
    _module("skopt", Optimizer=object)
    _module("skopt.space", Real=_Dim, Integer=_Dim, Categorical=_Dim)
    sys.path.insert(0, REF)


def describe_parser(parser):
    out = []
    for a in parser._actions:
        if isinstance(a, argparse._HelpAction):
            continue
        out.append({"option_strings": list(a.option_strings), "dest": a.dest, "default": a.default,
                    "type": getattr(a.type, "__name__", None), "action": type(a).__name__,
                    "choices": list(a.choices) if a.choices else None})
    return out


def main():
    install_stubs()
    import hyperparameter_search_option3 as opt3  # noqa: E402 (reference, under stubs)
    import mpiLAPI  # noqa: E402

    parser = opt3.make_parser()
    defaults = vars(parser.parse_args([]))
    space = [("nb_filters", 10, 50), ("pool_size", 2, 10), ("kernel_size", 2, 10), ("dense", 50, 200)]
    rng = np.random.RandomState(7)
    points = [[10, 2, 2, 50, 0.0], [50, 10, 10, 200, 1.0], [32, 2, 3, 128, 0.25]]
    for _ in range(7):
        points.append([int(rng.randint(lo, hi + 1)) for _, lo, hi in space] + [float(rng.uniform())])
    names = [n for n, _, _ in space] + ["dropout"]
    models = []
    for p in points:
        builder = opt3.BuilderFromFunction(mpiLAPI.test_mnist, [_Dim(0, 1, name=n) for n in names])
        CALLS.clear()
        json_str = builder.builder(*p)               # ModelFromJsonTF stand-in returns the JSON itself
        models.append({"params": p, "names": names, "calls": list(CALLS), "json": json_str})
    # the reference's test_mnist reads 'drop_out' (the space's 'dropout' never reaches it)
    CALLS.clear()
    json_do = mpiLAPI.test_mnist(nb_filters=20, pool_size=3, kernel_size=4, dense=60, drop_out=0.4)
    models.append({"params": [20, 3, 4, 60], "names": ["nb_filters", "pool_size", "kernel_size", "dense"],
                   "extra": {"drop_out": 0.4}, "calls": list(CALLS), "json": json_do})
    doc = {"generated_by": "tests/golden/make_reference_cli_mnist_fixture.py",
           "parser": describe_parser(parser), "defaults": defaults, "test_mnist": models}
    with open(OUT, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    print(f"wrote {OUT}: {len(doc['parser'])} flags, {len(models)} test_mnist models")


if __name__ == "__main__":
    main()
