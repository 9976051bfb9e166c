"""Model-builder plugin interface, drop-in for the reference's builders.

* ``test_mnist(**args) -> str`` -- /root/reference/mpiLAPI.py:138-176: the Keras
  MNIST ConvNet as a JSON string.  Keras is not available (nor needed): the
  JSON mirrors ``Sequential.to_json()`` (``class_name``/``config``/``layers``) and
  is what :func:`spec_from_json` ingests into a device :class:`TrialSpec`.
  The reference reads ``args.get('drop_out', 0.25)`` while its search space
  names the dimension ``dropout`` (option3:131): the dimension is dead and
  the rate stays 0.25 -- reproduced here.
* ``test_densenet`` -- mpiLAPI.py:197-201 (DenseNet) as a JSON spec that
  ingests into a :class:`DenseNetSpec` the DenseNet population engine
  (densenet.py) trains.  The topclass CNN and the 3-D GAN (mpiLAPI.py:178-195,
  option3:110-114, 144-168) are out of scope: their data and models
  are not in the BASELINE configs, so no builder is offered for them.
* ``BuilderFromFunction`` -- hyperparameter_search_option3.py:22-31: zips the
  named dimensions with a parameter list, calls ``model_fn(**named)`` and wraps
  the JSON in a ``ModelFromJson`` with settable ``comm`` / ``device`` and
  ``get_device_name`` (used by process_block.py:64-67).
* ``BaseModel`` / ``DenseNetModel`` -- base_model.py:8-19, 57-92:
  ``build(params) -> json``, ``get_parameter_grid()``, ``get_name()``.
"""
from __future__ import annotations

import json

import numpy as np

from .population import TrialSpec

KERAS_VERSION = "2.2.4"   # what the JSON claims to be; the content is all that is read


def _layer(cls, **cfg):
    return {"class_name": cls, "config": cfg}


def _sequential(layers, name="sequential_1"):
    return json.dumps({"class_name": "Sequential", "config": {"name": name, "layers": layers},
                       "keras_version": KERAS_VERSION, "backend": "tensorflow"})


def test_mnist(**args):
    """MNIST ConvNet from keras/examples/mnist_cnn.py (mpiLAPI.py:138-176)."""
    nb_classes = 10
    nb_filters = int(args.get("nb_filters", 32))
    ps = int(args.get("pool_size", 2))
    ks = int(args.get("kernel_size", 3))
    do = float(args.get("drop_out", 0.25))      # sic: the space's 'dropout' never reaches here
    dense = int(args.get("dense", 128))
    layers = [
        _layer("Conv2D", name="conv2d_1", filters=nb_filters, kernel_size=[ks, ks], strides=[1, 1],
               padding="valid", batch_input_shape=[None, 28, 28, 1], data_format="channels_last",
               activation="linear", use_bias=True, kernel_initializer="glorot_uniform",
               bias_initializer="zeros"),
        _layer("Activation", name="activation_1", activation="relu"),
        _layer("Conv2D", name="conv2d_2", filters=nb_filters, kernel_size=[ks, ks], strides=[1, 1],
               padding="valid", activation="linear", use_bias=True, kernel_initializer="glorot_uniform",
               bias_initializer="zeros"),
        _layer("Activation", name="activation_2", activation="relu"),
        _layer("MaxPooling2D", name="max_pooling2d_1", pool_size=[ps, ps], strides=[ps, ps], padding="valid"),
        _layer("Dropout", name="dropout_1", rate=do),
        _layer("Flatten", name="flatten_1"),
        _layer("Dense", name="dense_1", units=dense, activation="linear", use_bias=True,
               kernel_initializer="glorot_uniform", bias_initializer="zeros"),
        _layer("Activation", name="activation_3", activation="relu"),
        _layer("Dropout", name="dropout_2", rate=do),
        _layer("Dense", name="dense_2", units=nb_classes, activation="linear", use_bias=True,
               kernel_initializer="glorot_uniform", bias_initializer="zeros"),
        _layer("Activation", name="activation_4", activation="softmax"),
    ]
    return _sequential(layers)


def test_densenet(nb_classes=3, img_dim=(150, 94, 5), depth=10, nb_dense_block=3, growth_rate=12,
                  dropout_rate=0.00, nb_filter=16, lr=1e-3):
    """mpiLAPI.py:197-201: ``DenseNet(...)`` (densenet.py:135-196), compiled with
    ``Adam(lr)``, returned as ``to_json()`` -- the Keras functional-model JSON
    (:func:`mpi_opt_amd.keras_json.densenet_json`).  ``to_json`` carries no
    compile arguments, so ``lr`` does not reach the trainer (as in the reference)."""
    from .keras_json import densenet_json

    return densenet_json(nb_classes, img_dim, depth, nb_dense_block, growth_rate, nb_filter,
                         dropout_rate=dropout_rate)


class DenseNetSpec:
    """A DenseNet trial: the architecture (densenet.py:135) and its Adam lr, which
    the reference compiles into the model (base_model.py:67-71) and searches."""

    def __init__(self, arch, lr):
        self.arch = arch
        self.lr = float(lr)

    def flops_per_sample_train(self):
        from .densenet import flops_per_sample_train

        return flops_per_sample_train(self.arch.layers())


def spec_from_json(json_str, lr=1e-3, seed=0):
    """Ingest a Keras JSON into a device spec: the test_mnist Sequential topology
    -> :class:`TrialSpec`; a functional DenseNet ``Model`` (densenet.py's graph,
    from ``test_densenet`` / ``DenseNetModel.build`` or Keras itself) ->
    :class:`DenseNetSpec` trained with the trainer's ``lr``."""
    d = json.loads(json_str)
    if d.get("class_name") in ("Model", "Functional"):
        from .keras_json import densenet_arch_from_json

        arch, wd = densenet_arch_from_json(d)
        if abs(wd - 1e-4) > 1e-10:
            raise ValueError(f"DenseNet population trains weight_decay 1e-4 (densenet.py:136), JSON has {wd}")
        return DenseNetSpec(arch, lr)
    if d.get("class_name") != "Sequential":
        raise ValueError("population engine trains the test_mnist Sequential topology only")
    layers = d["config"]["layers"] if isinstance(d["config"], dict) else d["config"]
    kinds = [l["class_name"] for l in layers]
    expect = ["Conv2D", "Activation", "Conv2D", "Activation", "MaxPooling2D", "Dropout", "Flatten", "Dense",
              "Activation", "Dropout", "Dense", "Activation"]
    if kinds != expect:
        raise ValueError(f"unsupported topology {kinds}")
    c1, c2, pool, dr1, d1, dr2, d2 = (layers[i]["config"] for i in (0, 2, 4, 5, 7, 9, 10))
    F, k = int(c1["filters"]), int(c1["kernel_size"][0])
    shape = c1.get("batch_input_shape", [None, 28, 28, 1])
    if list(shape[1:]) != [28, 28, 1] or c1.get("padding", "valid") != "valid":
        raise ValueError("population engine expects 28x28x1 inputs and valid convolutions")
    if int(c2["filters"]) != F or int(c2["kernel_size"][0]) != k or int(d2["units"]) != 10:
        raise ValueError("unsupported test_mnist variant")
    if float(dr1["rate"]) != float(dr2["rate"]):
        raise ValueError("both dropout layers must share one rate")
    acts = [layers[i]["config"]["activation"] for i in (1, 3, 8, 11)]
    if acts != ["relu", "relu", "relu", "softmax"]:
        raise ValueError(f"unsupported activations {acts}")
    return TrialSpec(nb_filters=F, kernel_size=k, pool_size=int(pool["pool_size"][0]), dense=int(d1["units"]),
                     lr=lr, dropout=float(dr1["rate"]), seed=seed)


class ModelFromJson:
    """Stand-in for mpi_learn's ModelFromJsonTF (option3:27-31)."""

    def __init__(self, comm, json_str=None, device_name="cpu"):
        self.comm = comm
        self.json_str = json_str
        self.device = device_name

    def get_device_name(self, device):
        return device

    def spec(self, lr=1e-3, seed=0):
        return spec_from_json(self.json_str, lr=lr, seed=seed)


class BuilderFromFunction:
    """option3:22-31: builder(*params) -> ModelFromJson(model_fn(**named params))."""

    def __init__(self, model_fn, parameters):
        self.model_fn = model_fn
        self.parameters = parameters

    def builder(self, *params):
        args = dict(zip([p.name for p in self.parameters], params))
        return ModelFromJson(None, json_str=self.model_fn(**args))


class BaseModel:
    """base_model.py:8-19 interface."""

    def build(self, params):
        raise NotImplementedError

    def get_parameter_grid(self):
        raise NotImplementedError

    def get_name(self):
        raise NotImplementedError


class DenseNetModel(BaseModel):
    """base_model.py:57-92."""

    def __init__(self, input_shape=(150, 94, 5)):
        self.input_shape = input_shape

    def build(self, params):
        """base_model.py:62-73: the lr dimension (10**params[5]) is compiled into the
        model, which ``to_json`` drops -- the JSON carries the architecture only."""
        return test_densenet(nb_classes=3, img_dim=self.input_shape, depth=int(params[0]),
                             nb_dense_block=int(params[1]), growth_rate=int(params[2]), dropout_rate=float(params[3]),
                             nb_filter=int(params[4]), lr=10.0 ** params[5])

    def get_parameter_grid(self):
        return [(10, 10), (3, 3), (12, 12), (.0, .0), (16, 16), (-5, 1)]

    def get_name(self):
        return "DenseNet"


# --- search spaces of the reference examples --------------------------------
def mnist_space():
    """option3:126-133."""
    from .space import Integer, Real

    return [Integer(10, 50, name="nb_filters"), Integer(2, 10, name="pool_size"),
            Integer(2, 10, name="kernel_size"), Integer(50, 200, name="dense"),
            Real(0.0, 1.0, name="dropout")]


def flops_of_params(model_fn, names, params):
    spec = spec_from_json(model_fn(**dict(zip(names, params))))
    return spec.flops_per_sample_train()


__all__ = ["test_mnist", "test_densenet", "spec_from_json", "DenseNetSpec", "ModelFromJson", "BuilderFromFunction",
           "BaseModel", "DenseNetModel", "mnist_space"]
