"""Trial loader format: realtime-st-gcn_amd/data.py against the reference's own
prep_pkummd (data_prep/prep.py:14-48) and SkeletonDatasetFromDirectory (data_prep/dataset.py:88-125), pinned
by tests/golden/loader.npz (made by tests/golden/make_golden_loader.py from the reference).  The raw PKU-MMD-
shaped files are rebuilt here from the stored arrays exactly as the generator wrote them, so both sides read the
same bytes.

Divergences, each pinned explicitly below: prep.py:28 sizes the per-frame label vector by features.shape[0]
after the transpose (3, the channel count), so the reference writes 3 labels per trial; the restatement
writes L (what the loader and training need) and its first 3 entries equal the reference's.
"""
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "loader.npz"), allow_pickle=False)
N = len(G["names"])


@pytest.fixture(scope="module")
def data(pkg):
    return pkg.data


def write_raw(root):
    """Same bytes as make_golden_loader.write_raw (that module imports the reference, so it is not imported)."""
    fmt = str(G["fmt"])
    for sub in ("features", "labels", "train/features", "train/labels", "val/features", "val/labels"):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
    for i in range(N):
        n = str(G["names"][i])
        np.savetxt(os.path.join(root, "features", n + ".txt"), G["feat%d" % i], fmt=fmt)
        np.savetxt(os.path.join(root, "labels", n + ".txt"), G["rows%d" % i], fmt="%d", delimiter=",")
    with open(os.path.join(root, "cross-view.txt"), "w") as fo:
        fo.write("Training videos:\n" + ", ".join(str(t) for t in G["train"]) + ", \nValidataion videos:\n")


def test_prep_pkummd_matches_reference(data, tmp_path):
    root = str(tmp_path)
    write_raw(root)
    data.prep_pkummd(root)
    assert os.listdir(os.path.join(root, "features")) == [] and os.listdir(os.path.join(root, "labels")) == []
    for i in range(N):
        n, split = str(G["names"][i]), str(G["split%d" % i])
        assert os.path.exists(os.path.join(root, split, "features", n + ".npy")), (n, split)
        x = np.load(os.path.join(root, split, "features", n + ".npy"), allow_pickle=False)
        ref = G["npy%d" % i]
        assert x.dtype == ref.dtype == np.float32 and x.shape == ref.shape
        assert np.array_equal(x, ref), n  # bit-exact
        lab = np.loadtxt(os.path.join(root, split, "labels", n + ".csv"), delimiter=",")
        assert np.array_equal(lab, G["frames%d" % i]), n
        assert np.array_equal(lab[:3], G["csv%d" % i]), n  # the reference's 3-entry vector (prep.py:28)


def test_prep_pkummd_single_action_row(data, tmp_path):
    """A one-row action file (the reference's loadtxt gives a 1-D array there, prep.py:27-30)."""
    root = str(tmp_path)
    for sub in ("features", "labels"):
        os.makedirs(os.path.join(root, sub))
    np.savetxt(os.path.join(root, "features", "0001-L.txt"), np.ones((10, 150), np.float32), fmt="%.6f")
    np.savetxt(os.path.join(root, "labels", "0001-L.txt"), np.array([[4, 2, 6, 1]]), fmt="%d", delimiter=",")
    with open(os.path.join(root, "cross-view.txt"), "w") as fo:
        fo.write("Training videos:\n0001-L, \n")
    data.prep_pkummd(root)
    lab = np.loadtxt(os.path.join(root, "train", "labels", "0001-L.csv"), delimiter=",")
    assert lab.tolist() == [0, 0, 4, 4, 4, 4, 0, 0, 0, 0]


def test_prep_pkummd_split_like_reference(data, tmp_path):
    """prep.py:17 splits the train line on ", " without stripping: an id that ends the line (no trailing
    ", ") keeps its newline, never matches, and its trial lands in 'val' — reproduced, not 'fixed'."""
    root = str(tmp_path)
    for sub in ("features", "labels"):
        os.makedirs(os.path.join(root, sub))
    for n in ("0001-L", "0002-L"):
        np.savetxt(os.path.join(root, "features", n + ".txt"), np.ones((8, 150), np.float32), fmt="%.6f")
        np.savetxt(os.path.join(root, "labels", n + ".txt"), np.array([[4, 2, 6, 1], [3, 6, 8, 1]]), fmt="%d",
                   delimiter=",")
    with open(os.path.join(root, "cross-view.txt"), "w") as fo:
        fo.write("Training videos:\n0001-L, 0002-L\nValidation videos:\n")
    data.prep_pkummd(root)
    assert os.path.exists(os.path.join(root, "train", "features", "0001-L.npy"))
    assert os.path.exists(os.path.join(root, "val", "features", "0002-L.npy"))


def _dataset_dir(root):
    os.makedirs(os.path.join(root, "f"))
    os.makedirs(os.path.join(root, "l"))
    for i in range(N):
        n = str(G["names"][i])
        np.save(os.path.join(root, "f", n + ".npy"), G["npy%d" % i])
        np.savetxt(os.path.join(root, "l", n + ".csv"), G["frames%d" % i], delimiter=",")
    with open(os.path.join(root, "actions.txt"), "w") as fo:
        fo.write("\n".join("action%d" % k for k in range(int(G["nclass"]))))
    return os.path.join(root, "f"), os.path.join(root, "l"), os.path.join(root, "actions.txt")


def test_dataset_matches_reference(data, tmp_path):
    ds = data.SkeletonDatasetFromDirectory(*_dataset_dir(str(tmp_path)))
    assert len(ds) == int(G["len"]) == N
    assert len(ds.actions) == int(G["nclass"]) and ds.actions[1] == "action0"
    for i in range(N):
        x, y = ds[i]
        assert x.dtype == torch.float32 and y.dtype == torch.int64
        assert torch.equal(x, torch.from_numpy(G["item_x%d" % i]))
        assert torch.equal(y, torch.from_numpy(G["item_y%d" % i]))
    dist = ds.__get_distribution__("cpu")
    assert dist.dtype == torch.float32
    assert torch.equal(dist, torch.from_numpy(G["distribution"]))


def test_dataset_through_dataloader(data, tmp_path):
    """batch_size=1 DataLoader as the reference's processor builds it (processor.py:160-173)."""
    ds = data.SkeletonDatasetFromDirectory(*_dataset_dir(str(tmp_path)))
    seen = 0
    for x, y in torch.utils.data.DataLoader(ds, batch_size=1, shuffle=False):
        assert x.shape[:2] == (1, 3) and x.shape[3] == 25 and y.shape == (1, x.shape[2])
        seen += 1
    assert seen == N


@pytest.mark.gpu
def test_dataset_device_staging(data, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ds = data.SkeletonDatasetFromDirectory(*_dataset_dir(str(tmp_path)), device="cuda:0")
    x, y = ds[2]
    torch.cuda.synchronize()
    assert x.is_cuda and y.is_cuda
    assert torch.equal(x.cpu(), torch.from_numpy(G["item_x2"]))
    assert torch.equal(y.cpu(), torch.from_numpy(G["item_y2"]))
    assert torch.equal(ds.__get_distribution__("cuda:0").cpu(), torch.from_numpy(G["distribution"]))
