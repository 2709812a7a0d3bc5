"""Parallel host decoding of the drop-in data loader (data_loader.content_style_iter / content_iter,
the reference's DataLoader(num_workers=4 | 8) in train.py:66-75 and train_autoencoder.py:188-195):
worker processes decode, the trainer process applies the transform. CPU only: the transform here is
a host stand-in for the device ToTensor (the device transforms are tests/test_gpu_augment.py's)."""
import numpy as np
import pytest
import torch
from PIL import Image

from arbitrarystyletransfer_amd import data_loader as DL


def _write_images(d, n, seed, size=(12, 10)):
    d.mkdir()
    rng = np.random.default_rng(seed)
    arrs = []
    for i in range(n):
        a = rng.integers(0, 256, (size[1], size[0], 3), dtype=np.uint8)
        Image.fromarray(a).save(d / f"img{i}.png")
        arrs.append(a)
    return arrs


def _host_to_tensor(arr):
    assert isinstance(arr, np.ndarray) and arr.dtype == np.uint8 and arr.ndim == 3
    return torch.from_numpy(arr.copy()).permute(2, 0, 1).float() / 255.0


def _find(t, arrs):
    a = (t.permute(1, 2, 0) * 255.0).round().to(torch.uint8).numpy()
    return [i for i, r in enumerate(arrs) if np.array_equal(r, a)]


@pytest.mark.parametrize("workers", [0, 2])
def test_content_style_iter_decodes_in_workers(tmp_path, workers):
    content = _write_images(tmp_path / "content", 5, 1)
    style = _write_images(tmp_path / "style", 4, 2)
    it = DL.content_style_iter([str(tmp_path / "content")], [str(tmp_path / "style")], _host_to_tensor,
                               batch_size=3, num_workers=workers)
    for _ in range(3):
        c, s = next(it)
        assert c.shape == (3, 3, 10, 12) and s.shape == (3, 3, 10, 12) and c.dtype == torch.float32
        for k in range(3):   # every image is one of the files, content from content, style from style
            assert len(_find(c[k], content)) == 1 and len(_find(s[k], style)) == 1


def test_content_iter_ae_and_bad_file_retry(tmp_path, capsys):
    content = _write_images(tmp_path / "content", 3, 3)
    (tmp_path / "content" / "broken.png").write_bytes(b"not an image")
    it = DL.content_iter([str(tmp_path / "content")], _host_to_tensor, batch_size=4, num_workers=2)
    for _ in range(4):
        b = next(it)
        assert b.shape == (4, 3, 10, 12)
        for k in range(4):   # the unreadable file is skipped by a retry (data_loader.py:190-192)
            assert len(_find(b[k], content)) == 1


def test_host_decoded_matches_dataset_item(tmp_path):
    """The worker's decode is the dataset's own _get_item minus the transform: same RNG draws."""
    _write_images(tmp_path / "content", 4, 4)
    _write_images(tmp_path / "style", 4, 5)
    ds = DL.FlatFolderDataset([str(tmp_path / "content")], [str(tmp_path / "style")], transform=None)
    torch.manual_seed(7)
    c1, s1 = DL.HostDecoded(ds)[0]
    torch.manual_seed(7)
    c2, s2 = ds[0]
    assert np.array_equal(c1, np.asarray(c2)) and np.array_equal(s1, np.asarray(s2))


def test_spawned_workers_after_gpu_init(tmp_path, monkeypatch):
    """A caller that initialised the GPU before building the iterator gets spawned workers
    (data_loader._decoded_loader): HostDecoded and the dataset pickle into a fresh interpreter that
    imports the package and decodes with PIL only. The GPU init is stubbed (CPU host)."""
    content = _write_images(tmp_path / "content", 3, 6)
    monkeypatch.setattr(DL, "_gpu_initialized", lambda: True)
    seen = {}
    orig = DL.data.DataLoader

    def spy(*a, **kw):
        seen["ctx"] = kw.get("multiprocessing_context")
        return orig(*a, **kw)
    monkeypatch.setattr(DL.data, "DataLoader", spy)
    it = DL.content_iter([str(tmp_path / "content")], _host_to_tensor, batch_size=2, num_workers=1)
    assert seen["ctx"] == "spawn"
    b = next(it)
    assert b.shape == (2, 3, 10, 12)
    for k in range(2):
        assert len(_find(b[k], content)) == 1
