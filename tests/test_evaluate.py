"""The torchvision-free evaluation harness (data_free_quantization_amd/evaluate.py),
main_dfq.py:66-113's inference_all.  CPU only: synthetic ImageFolder / VOC trees
written with PIL, hand-computed expectations.  (torchvision and the reference's
dataset code are absent, so the transforms are checked against their published
arithmetic, not against those libraries: parity unpinned.)"""
from pathlib import Path

import numpy as np
import pytest
import torch

from data_free_quantization_amd import evaluate as E

Image = pytest.importorskip("PIL.Image")


def _img(w, h, rgb):
    return Image.fromarray(np.full((h, w, 3), rgb, dtype=np.uint8))


def _folder(tmp_path):
    root = tmp_path / "val"
    for cls, rgb in (("n01_red", (250, 10, 10)), ("n02_blue", (10, 10, 250))):
        (root / cls).mkdir(parents=True)
        for k, (w, h) in enumerate(((300, 260), (224, 400), (512, 512))):
            _img(w, h, rgb).save(root / cls / f"img{k}.png")
    (root / "n01_red" / "notes.txt").write_text("not an image")
    return root


def test_image_folder_order_and_labels(tmp_path):
    ds = E.ImageFolder(str(_folder(tmp_path)))
    assert ds.classes == ["n01_red", "n02_blue"]
    assert [t for _, t in ds.samples] == [0, 0, 0, 1, 1, 1]
    assert [p.rsplit("/", 1)[1] for p, _ in ds.samples[:3]] == ["img0.png", "img1.png", "img2.png"]
    x, y = ds[0]
    assert x.shape == (3, 224, 224) and x.dtype == torch.float32 and y == 0


def test_cls_transform_sizes_and_normalisation():
    # shorter side -> 256 (long side int(256 * long / short)), centre 224 crop
    assert E.resize_shorter(_img(300, 260, (0, 0, 0)), 256).size == (int(256 * 300 / 260), 256)
    assert E.resize_shorter(_img(224, 400, (0, 0, 0)), 256).size == (256, int(256 * 400 / 224))
    img = Image.fromarray(np.arange(295 * 256 * 3, dtype=np.uint32).astype(np.uint8).reshape(256, 295, 3))
    c = E.center_crop(img, 224)
    top, left = int(round((256 - 224) / 2.0)), int(round((295 - 224) / 2.0))
    assert np.array_equal(np.asarray(c), np.asarray(img)[top:top + 224, left:left + 224])
    x = E.cls_transform(_img(300, 260, (200, 100, 50)))
    for ch, v in enumerate((200, 100, 50)):
        expect = (torch.tensor(v / 255.0, dtype=torch.float32) - E.MEAN[ch]) / E.STD[ch]
        assert torch.all(x[ch] == expect)


def test_evaluator_confusion_and_miou():
    ev = E.Evaluator(3)
    gt = np.array([[0, 0, 1, 1], [2, 2, 255, 1]])
    pred = np.array([[0, 1, 1, 1], [2, 0, 2, 1]])
    ev.add_batch(gt, pred)
    assert ev.confusion.tolist() == [[1, 1, 0], [0, 3, 0], [1, 0, 1]]
    iou = [1 / (2 + 2 - 1), 3 / (3 + 4 - 3), 1 / (2 + 1 - 1)]
    assert ev.mean_iou() == pytest.approx(np.mean(iou))
    assert ev.pixel_accuracy() == pytest.approx(5 / 7)


def test_fix_scale_crop():
    img = _img(600, 400, (1, 2, 3))
    lab = np.zeros((400, 600), dtype=np.uint8)
    lab[:, 300:] = 7
    lab[0, 0] = 255
    i2, m2 = E.fix_scale_crop(img, Image.fromarray(lab), 200)
    assert i2.size == (200, 200) and m2.size == (200, 200)
    assert set(np.unique(np.asarray(m2)).tolist()) <= {0, 7, 255}   # nearest: no new labels


class _ColourNet(torch.nn.Module):
    """Predicts class 0 when red dominates, 1 otherwise (per image)."""

    def forward(self, x):
        r, b = x[:, 0].mean((1, 2)), x[:, 2].mean((1, 2))
        return torch.stack([r - b, b - r], 1)


def test_inference_cls_end_to_end(tmp_path):
    acc = E.inference_cls(_ColourNet(), str(_folder(tmp_path)), device="cpu", batch_size=4, workers=0)
    assert acc == 1.0


def test_inference_seg_end_to_end(tmp_path):
    base = tmp_path / "VOCdevkit" / "VOC2012"
    for d in ("ImageSets/Segmentation", "JPEGImages", "SegmentationClass"):
        (base / d).mkdir(parents=True)
    ids = []
    for k in range(3):
        arr = np.zeros((80, 100, 3), dtype=np.uint8)
        lab = np.zeros((80, 100), dtype=np.uint8)
        arr[:, 50:, 0] = 255          # red right half = class 15
        lab[:, 50:] = 15
        lab[0, :] = 255               # ignored border
        Image.fromarray(arr).save(base / "JPEGImages" / f"im{k}.jpg", quality=100)
        Image.fromarray(lab).save(base / "SegmentationClass" / f"im{k}.png")
        ids.append(f"im{k}")
    (base / "ImageSets" / "Segmentation" / "val.txt").write_text("\n".join(ids) + "\n")

    class _Seg(torch.nn.Module):
        def forward(self, x):
            red = (x[:, 0] > 0.5).float()
            out = torch.zeros(x.shape[0], 21, *x.shape[2:])
            out[:, 15] = red
            out[:, 0] = 1 - red
            return out

    miou = E.inference_seg(_Seg(), str(base), device="cpu", batch_size=2, workers=0, crop_size=64)
    assert miou > 0.9


def test_seg_transform_matches_reference_fixture():
    """FixScaleCrop -> Normalize -> ToTensor (the reference's VOC validation
    transform, dataset_utils/segmentation/pascal.py:108-112) on seeded images and
    masks: image and label tensors bit-exact with the reference's own output
    (tests/golden/seg_transforms.npz, make_golden.py seg)."""
    import json
    from PIL import Image
    from data_free_quantization_amd.evaluate import seg_transform
    z = np.load(Path(__file__).resolve().parent / "golden" / "seg_transforms.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    assert len(meta["cases"]) >= 6
    for i, c in enumerate(meta["cases"]):
        out = seg_transform(Image.fromarray(z[f"img{i}"]), Image.fromarray(z[f"mask{i}"]), c["crop"])
        img, lab = out["image"].numpy(), out["label"].numpy()
        assert img.dtype == np.float32 and img.shape == (3, c["crop"], c["crop"]), (i, c)
        assert np.array_equal(img.view(np.uint32), z[f"out_img{i}"].view(np.uint32)), (i, c)
        assert np.array_equal(lab, z[f"out_label{i}"]) and lab.dtype == z[f"out_label{i}"].dtype, (i, c)
