"""Write the HDF5 fixtures that pin mpi_opt_amd/h5.py (the build's own HDF5
reader) -- run with an interpreter that has h5py (here: /opt/conda/bin/python3.9,
h5py 3.3.0 / HDF5 1.10.6; the product interpreter has no h5py):

    env -u PYTHONPATH /opt/conda/bin/python3.9 tests/golden/make_h5_fixtures.py

The files mimic what the reference's mpi_learn ``H5Data(features_name='features',
labels_name='labels')`` reads for the mnist example (hyperparameter_search_option3.py:
134-142, 253-259): one ``features`` and one ``labels`` dataset per file.  They cover
the layouts h5py produces: superblock v0 / object header v1 / symbol-table root
(libver 'earliest') and superblock v3 / object header v2 / compact links (libver
'latest'); contiguous, compact and chunked storage; gzip + shuffle + fletcher32
filters; B-tree v1, single-chunk, implicit and fixed-array chunk indexes; little- and
big-endian, float / integer types.  Expected arrays are stored next to them in
h5_expected.npz.
"""
import os

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "h5")


def mnist_like(n, seed, onehot=True):
    rng = np.random.RandomState(seed)
    x = rng.uniform(size=(n, 28, 28, 1)).astype(np.float32)
    lab = rng.randint(0, 10, size=n)
    y = np.eye(10, dtype=np.float32)[lab] if onehot else lab.astype(np.int64)
    return x, y


def main():
    os.makedirs(OUT, exist_ok=True)
    exp = {}

    def put(name, arrays):
        for k, v in arrays.items():
            exp[f"{name}/{k}"] = v

    # 1. h5py defaults (libver earliest): contiguous float32 features, one-hot labels
    x, y = mnist_like(40, 1)
    with h5py.File(os.path.join(OUT, "mnist_a.h5"), "w", libver="earliest") as f:
        f.create_dataset("features", data=x)
        f.create_dataset("labels", data=y)
    put("mnist_a.h5", {"features": x, "labels": y})

    # 2. earliest + chunked / gzip + shuffle (B-tree v1 chunk index), int labels, ragged last chunk
    x, y = mnist_like(37, 2, onehot=False)
    with h5py.File(os.path.join(OUT, "mnist_b.h5"), "w", libver="earliest") as f:
        f.create_dataset("features", data=x, chunks=(8, 28, 28, 1), compression="gzip", shuffle=True)
        f.create_dataset("labels", data=y, chunks=(16,), compression="gzip")
    put("mnist_b.h5", {"features": x, "labels": y})

    # 3. libver latest: object header v2, fixed-array chunk index, fletcher32; flat features
    x, y = mnist_like(50, 3)
    x = x.reshape(50, 784)
    with h5py.File(os.path.join(OUT, "mnist_c.h5"), "w", libver="latest") as f:
        f.create_dataset("features", data=x, chunks=(10, 784), compression="gzip", fletcher32=True)
        f.create_dataset("labels", data=y, chunks=(50, 10))       # single-chunk index
        f.create_dataset("extra", data=np.arange(5, dtype=">i4"))    # big-endian, contiguous
    put("mnist_c.h5", {"features": x, "labels": y, "extra": np.arange(5, dtype=np.int32)})

    # 4. latest, compact storage and float64 / uint8, implicit chunk index (no filters,
    #    early allocation)
    feats = (np.random.RandomState(4).uniform(size=(6, 28, 28, 1)) * 255).astype(np.uint8)
    labs = np.array([3, 1, 4, 1, 5, 9], dtype=np.float64)
    with h5py.File(os.path.join(OUT, "mnist_d.h5"), "w", libver="latest") as f:
        dcpl = h5py.h5p.create(h5py.h5p.DATASET_CREATE)
        dcpl.set_layout(h5py.h5d.COMPACT)
        sp = h5py.h5s.create_simple(labs.shape)
        h5py.h5d.create(f.id, b"labels", h5py.h5t.IEEE_F64LE, sp, dcpl).write(h5py.h5s.ALL, h5py.h5s.ALL, labs)
        dcpl2 = h5py.h5p.create(h5py.h5p.DATASET_CREATE)
        dcpl2.set_chunk((2, 28, 28, 1))
        dcpl2.set_alloc_time(h5py.h5d.ALLOC_TIME_EARLY)
        sp2 = h5py.h5s.create_simple(feats.shape)
        h5py.h5d.create(f.id, b"features", h5py.h5t.STD_U8LE, sp2, dcpl2).write(h5py.h5s.ALL, h5py.h5s.ALL, feats)
    put("mnist_d.h5", {"features": feats, "labels": labs})

    np.savez(os.path.join(HERE, "h5_expected.npz"), **exp)
    for fn in sorted(os.listdir(OUT)):
        print(fn, os.path.getsize(os.path.join(OUT, fn)))


if __name__ == "__main__":
    main()
