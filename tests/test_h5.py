"""The build's HDF5 reader (mpi_opt_amd/h5.py) against files written by h5py 3.3
/ HDF5 1.10.6 (tests/golden/make_h5_fixtures.py): every dataset reads back
bit-identical across superblock v0/v3, object header v1/v2, contiguous / compact /
chunked storage, B-tree v1 / single-chunk / implicit / fixed-array chunk indexes,
gzip / shuffle / fletcher32 filters and both byte orders."""
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN

H5DIR = os.path.join(GOLDEN, "h5")
EXP = np.load(os.path.join(GOLDEN, "h5_expected.npz"))


@pytest.mark.parametrize("key", sorted(EXP.files))
def test_dataset_reads_back_bit_identical(key):
    from mpi_opt_amd.h5 import H5File

    fn, ds = key.split("/")
    f = H5File(os.path.join(H5DIR, fn))
    got = f[ds].read()
    want = EXP[key]
    assert got.shape == want.shape and got.dtype == want.dtype.newbyteorder("=")
    assert np.array_equal(got, want)


def test_keys_and_errors(tmp_path):
    from mpi_opt_amd.h5 import H5Error, H5File

    f = H5File(os.path.join(H5DIR, "mnist_c.h5"))
    assert sorted(f.keys()) == ["extra", "features", "labels"]
    with pytest.raises(KeyError):
        f["nope"]
    bad = tmp_path / "x.h5"
    bad.write_bytes(b"not hdf5" * 100)
    with pytest.raises(H5Error):
        H5File(str(bad))


def test_load_xy_and_option3_split(tmp_path):
    """features -> [n, 784] float32, one-hot or integer labels -> class ids; the
    first 70 % of the files train, the rest validate (option3:134-139)."""
    import shutil

    from mpi_opt_amd.h5 import load_xy, split_files

    for fn in ("mnist_a.h5", "mnist_b.h5", "mnist_c.h5"):
        shutil.copy(os.path.join(H5DIR, fn), tmp_path / fn)
    tr, va = split_files(str(tmp_path))
    assert [os.path.basename(p) for p in tr] == ["mnist_a.h5", "mnist_b.h5"]
    assert [os.path.basename(p) for p in va] == ["mnist_c.h5"]
    x, y = load_xy(tr + va)
    assert x.shape == (40 + 37 + 50, 784) and x.dtype == np.float32 and y.dtype == np.int32
    np.testing.assert_array_equal(x[:40], EXP["mnist_a.h5/features"].reshape(40, 784))
    np.testing.assert_array_equal(y[:40], EXP["mnist_a.h5/labels"].argmax(1))
    np.testing.assert_array_equal(y[40:77], EXP["mnist_b.h5/labels"])


def test_kfold_holdout_split():
    """n_fold 1: train = the train_list samples, validation = the val_list ones;
    n_fold > 1: contiguous KFold over the train_list samples only."""
    from mpi_opt_amd.population import kfold_split

    tr, va = kfold_split(127, 1, 0, holdout=77)
    assert tr.tolist() == list(range(77)) and va.tolist() == list(range(77, 127))
    tr, va = kfold_split(127, 5, 1, holdout=77)
    assert va.tolist() == list(range(16, 32)) and len(tr) == 77 - 16 and max(tr) == 76
    # synthetic data keeps option3's 70 % cut
    tr, va = kfold_split(100, 1, 0)
    assert len(tr) == 70 and len(va) == 30


def test_split_files_rejects_an_empty_side(tmp_path):
    """One file: 70 % of it is no training file -- a clear H5Error, not a numpy
    concatenate failure deep inside load_xy."""
    import shutil

    from mpi_opt_amd.h5 import H5Error, split_files

    shutil.copy(os.path.join(H5DIR, "mnist_a.h5"), tmp_path / "mnist_a.h5")
    with pytest.raises(H5Error, match="both need at least one"):
        split_files(str(tmp_path))
