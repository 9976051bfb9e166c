"""Generate tests/golden/densenet_keras_functional.json by running the
reference's own graph builder, /root/reference/densenet.py ``DenseNet(...)``,
against a minimal recording stand-in for the Keras 2.0/2.1 layer API (Keras is
not installed anywhere here).  The layer sequence, arguments and connectivity
in the fixture are therefore what densenet.py:12-196 itself calls; this script
only serialises them the way Keras 2.1's ``Model.to_json()`` does (Keras-1
keywords mapped by Keras 2's legacy interface: init -> kernel_initializer,
border_mode -> padding, bias -> use_bias, W_/b_regularizer ->
kernel_/bias_regularizer, dim_ordering "tf" -> data_format "channels_last",
BatchNormalization's mode=0 dropped; ``merge(mode='concat')`` -> the legacy
``Merge`` layer).

Run in the build container (needs /root/reference):
    python tests/golden/make_keras_densenet_fixture.py
The reference is only read here, never at test time.
"""
import json
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "densenet_keras_functional.json")
COUNTS = {}
CREATED = []


def _snake(cls):
    out = ""
    for i, ch in enumerate(cls):
        if ch.isupper() and i and (cls[i - 1].islower() or cls[i - 1].isdigit()):
            out += "_"
        out += ch.lower()
    return out


class Tensor:
    def __init__(self, layer):
        self.layer = layer


def _l2cfg(r):
    # Keras keeps regularizer factors as K.cast_to_floatx (float32): 1e-4 -> 9.999999747378752e-05
    return None if r is None else {"class_name": "L1L2", "config": {"l1": 0.0, "l2": float(np.float32(r))}}


INITS = {"he_uniform": {"class_name": "VarianceScaling",
                        "config": {"scale": 2.0, "mode": "fan_in", "distribution": "uniform", "seed": None}},
         "glorot_uniform": {"class_name": "VarianceScaling",
                            "config": {"scale": 1.0, "mode": "fan_avg", "distribution": "uniform", "seed": None}}}


class Layer:
    cls = None
    keras_base = None

    def __init__(self, name=None, **cfg):
        base = self.keras_base or _snake(self.cls)
        if name is None:
            COUNTS[base] = COUNTS.get(base, 0) + 1
            name = f"{base}_{COUNTS[base]}"
        self.name, self.cfg, self.inbound = name, cfg, None
        CREATED.append(self)

    def __call__(self, x):
        xs = x if isinstance(x, list) else [x]
        self.inbound = [t.layer.name for t in xs]
        return Tensor(self)

    def config(self):
        return {"name": self.name, "trainable": True, **self.cfg}


def Input(shape):
    l = Layer.__new__(Layer)
    l.cls = "InputLayer"
    COUNTS["input"] = COUNTS.get("input", 0) + 1
    l.name = f"input_{COUNTS['input']}"
    l.cfg = {"batch_input_shape": [None, *shape], "dtype": "float32", "sparse": False}
    l.inbound = []
    CREATED.append(l)
    return Tensor(l)


class Convolution2D(Layer):
    cls, keras_base = "Conv2D", "conv2d"

    def __init__(self, nb_filter, kernel, init="glorot_uniform", border_mode="valid", bias=True,
                 W_regularizer=None, name=None):
        super().__init__(name=name, filters=nb_filter, kernel_size=list(kernel), strides=[1, 1], padding=border_mode,
                         data_format="channels_last", dilation_rate=[1, 1], activation="linear", use_bias=bias,
                         kernel_initializer=INITS[init], bias_initializer={"class_name": "Zeros", "config": {}},
                         kernel_regularizer=_l2cfg(W_regularizer), bias_regularizer=None, activity_regularizer=None,
                         kernel_constraint=None, bias_constraint=None)


class BatchNormalization(Layer):
    cls, keras_base = "BatchNormalization", "batch_normalization"

    def __init__(self, mode=0, axis=-1, gamma_regularizer=None, beta_regularizer=None, name=None):
        assert mode == 0
        z, o = {"class_name": "Zeros", "config": {}}, {"class_name": "Ones", "config": {}}
        super().__init__(name=name, axis=axis, momentum=0.99, epsilon=0.001, center=True, scale=True,
                         beta_initializer=z, gamma_initializer=o, moving_mean_initializer=z,
                         moving_variance_initializer=o, beta_regularizer=_l2cfg(beta_regularizer),
                         gamma_regularizer=_l2cfg(gamma_regularizer), beta_constraint=None, gamma_constraint=None)


class Activation(Layer):
    cls = "Activation"

    def __init__(self, activation, name=None):
        super().__init__(name=name, activation=activation)


class Dropout(Layer):
    cls = "Dropout"

    def __init__(self, rate, name=None):
        super().__init__(name=name, rate=rate, noise_shape=None, seed=None)


class AveragePooling2D(Layer):
    cls, keras_base = "AveragePooling2D", "average_pooling2d"

    def __init__(self, pool_size, strides=None, name=None):
        super().__init__(name=name, pool_size=list(pool_size), padding="valid", strides=list(strides or pool_size),
                         data_format="channels_last")


class GlobalAveragePooling2D(Layer):
    cls, keras_base = "GlobalAveragePooling2D", "global_average_pooling2d"

    def __init__(self, dim_ordering="tf", name=None):
        super().__init__(name=name, data_format="channels_last" if dim_ordering == "tf" else "channels_first")


class Dense(Layer):
    cls = "Dense"

    def __init__(self, units, activation="linear", W_regularizer=None, b_regularizer=None, name=None):
        super().__init__(name=name, units=units, activation=activation, use_bias=True,
                         kernel_initializer=INITS["glorot_uniform"],
                         bias_initializer={"class_name": "Zeros", "config": {}},
                         kernel_regularizer=_l2cfg(W_regularizer), bias_regularizer=_l2cfg(b_regularizer),
                         activity_regularizer=None, kernel_constraint=None, bias_constraint=None)


class Merge(Layer):
    cls = "Merge"

    def __init__(self, mode, concat_axis, name=None):
        super().__init__(name=name, mode=mode, mode_type="raw", concat_axis=concat_axis, dot_axes=-1,
                         output_shape=None, output_shape_type="raw", output_mask=None, output_mask_type="raw",
                         arguments={})


def merge(inputs, mode="sum", concat_axis=-1):
    return Merge(mode, concat_axis)(inputs)


class Model:
    def __init__(self, input, output, name=None):
        self.inputs, self.outputs, self.name = input, output, name

    def to_json(self):
        layers = [{"name": l.name, "class_name": l.cls, "config": l.config(),
                   "inbound_nodes": [[[i, 0, 0, {}] for i in l.inbound]] if l.inbound else []} for l in CREATED]
        return json.dumps({"class_name": "Model", "config": {
            "name": self.name, "layers": layers, "input_layers": [[t.layer.name, 0, 0] for t in self.inputs],
            "output_layers": [[t.layer.name, 0, 0] for t in self.outputs]},
            "keras_version": "2.1.6", "backend": "tensorflow"}, indent=1)


def install_stub_keras(root):
    mods = {
        "keras": {}, "keras.models": {"Model": Model},
        "keras.layers": {"Input": Input, "merge": merge, "Permute": None},
        "keras.layers.core": {"Dense": Dense, "Dropout": Dropout, "Activation": Activation},
        "keras.layers.convolutional": {"Convolution2D": Convolution2D},
        "keras.layers.pooling": {"AveragePooling2D": AveragePooling2D,
                                 "GlobalAveragePooling2D": GlobalAveragePooling2D},
        "keras.layers.normalization": {"BatchNormalization": BatchNormalization},
        "keras.regularizers": {"l2": lambda v: v},
        "keras.backend": {"image_dim_ordering": lambda: "tf"},
    }
    for name, attrs in mods.items():
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        m.__path__ = []
        sys.modules[name] = m
    for name in mods:
        if "." in name:
            parent, child = name.rsplit(".", 1)
            setattr(sys.modules[parent], child, sys.modules[name])


def main():
    install_stub_keras(tempfile.mkdtemp())
    sys.path.insert(0, REF)
    import densenet  # /root/reference/densenet.py

    # BASELINE configs[4]: CIFAR-10 shape with the base_model.py:84-92 grid architecture
    m = densenet.DenseNet(nb_classes=10, img_dim=(32, 32, 3), depth=10, nb_dense_block=3, growth_rate=12,
                          nb_filter=16, dropout_rate=0.0, weight_decay=1e-4)
    with open(OUT, "w") as f:
        f.write(m.to_json())
    print(f"wrote {OUT}: {len(CREATED)} layers")


if __name__ == "__main__":
    main()
