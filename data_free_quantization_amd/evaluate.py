"""Evaluation harness of main_dfq (``inference_all``, main_dfq.py:66-113) without
torchvision: ImageNet-style ImageFolder top-1 and PASCAL VOC mIoU.

The reference evaluates classification with ``torchvision.datasets.ImageFolder``
+ ``Resize(256) / CenterCrop(224) / ToTensor / Normalize`` and a DataLoader of
256 (main_dfq.py:71-78,91-113), and segmentation with ``VOCSegmentation`` +
``forward_all`` (main_dfq.py:80-89) from ``dataset/`` and ``utils/segmentation/``,
which the reference tree does not contain.  torchvision is not installed here, so
this module restates those steps on PIL + numpy:

* ``ImageFolder``: classes = sorted sub-directories, samples sorted by path,
  torchvision's image extensions (torchvision/datasets/folder.py semantics);
* ``cls_transform``: shorter side to 256 with PIL bilinear (what torchvision's
  Resize does to a PIL image), centre crop 224 with torchvision's rounding,
  /255, per-channel normalisation;
* ``VOCSegmentation`` (split files under ImageSets/Segmentation, JPEGImages,
  SegmentationClass): the DeepLab codebase's validation transform, FixScaleCrop
  (shorter side to the crop size, bilinear image / nearest mask, centre crop)
  then the same normalisation;
* ``Evaluator`` / ``forward_all``: confusion matrix over the 21 classes
  (label 255 ignored), pixel accuracy and mean IoU.

Parity: the segmentation transform (FixScaleCrop, Normalize, ToTensor) is pinned
bit-exact to the reference's own custom_transforms.py (importable in the dev
container; fixtures tests/golden/seg_transforms.npz).  The classification path
stays "parity unpinned": torchvision (its Resize / CenterCrop / Normalize and
ImageFolder) is not installed here, so those are restatements of its published
behaviour, checked in tests/test_evaluate.py on hand-computed cases.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def _pil():
    from PIL import Image
    return Image


class ImageFolder(torch.utils.data.Dataset):
    """root/<class>/<image>: (tensor, class index), classes in sorted order."""

    def __init__(self, root: str, transform=None):
        self.classes = sorted(e.name for e in os.scandir(root) if e.is_dir())
        if not self.classes:
            raise FileNotFoundError(f"no class folders under {root}")
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.samples: List[Tuple[str, int]] = []
        for c in self.classes:
            for dirpath, _, files in sorted(os.walk(os.path.join(root, c), followlinks=True)):
                for f in sorted(files):
                    if f.lower().endswith(IMG_EXTENSIONS):
                        self.samples.append((os.path.join(dirpath, f), self.class_to_idx[c]))
        if not self.samples:
            raise FileNotFoundError(f"no images under {root}")
        self.transform = transform or cls_transform

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        path, target = self.samples[i]
        with open(path, "rb") as f:
            img = _pil().open(f).convert("RGB")
        return self.transform(img), target


def _normalize(arr: np.ndarray) -> torch.Tensor:
    """HWC uint8 -> CHW float32 (x / 255 - mean) / std."""
    x = torch.from_numpy(np.array(arr, dtype=np.uint8, copy=True)).permute(2, 0, 1).float().div(255.0)
    mean = torch.tensor(MEAN, dtype=torch.float32).view(3, 1, 1)
    std = torch.tensor(STD, dtype=torch.float32).view(3, 1, 1)
    return (x - mean) / std


def resize_shorter(img, size: int, resample=None):
    """torchvision Resize(int) on a PIL image: the shorter side becomes ``size``,
    the longer int(size * long / short)."""
    Image = _pil()
    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    if short == size:
        return img
    new_long = int(size * long / short)
    ow, oh = (size, new_long) if w <= h else (new_long, size)
    return img.resize((ow, oh), Image.BILINEAR if resample is None else resample)


def center_crop(img, size: int):
    """torchvision CenterCrop: top = int(round((h - size) / 2)), same for left
    (the image is at least ``size`` on both sides here)."""
    w, h = img.size
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return img.crop((left, top, left + size, top + size))


def cls_transform(img) -> torch.Tensor:
    """Resize(256), CenterCrop(224), ToTensor, Normalize (main_dfq.py:71-77)."""
    return _normalize(np.asarray(center_crop(resize_shorter(img, 256), 224), dtype=np.uint8))


class VOCSegmentation(torch.utils.data.Dataset):
    """PASCAL VOC 2012 segmentation split (base_dir = VOCdevkit/VOC2012)."""
    NUM_CLASSES = 21

    def __init__(self, base_size: int = 513, crop_size: int = 513, base_dir: str = "./VOCdevkit/VOC2012/",
                 split: str = "val"):
        self.crop_size = crop_size
        self.base_size = base_size
        with open(os.path.join(base_dir, "ImageSets", "Segmentation", split + ".txt")) as f:
            ids = [ln.strip() for ln in f if ln.strip()]
        self.images = [os.path.join(base_dir, "JPEGImages", i + ".jpg") for i in ids]
        self.labels = [os.path.join(base_dir, "SegmentationClass", i + ".png") for i in ids]
        for p in self.images + self.labels:
            if not os.path.isfile(p):
                raise FileNotFoundError(p)

    def __len__(self):
        return len(self.images)

    def __getitem__(self, i):
        Image = _pil()
        img = Image.open(self.images[i]).convert("RGB")
        mask = Image.open(self.labels[i])
        return seg_transform(img, mask, self.crop_size)


def fix_scale_crop(img, mask, crop: int):
    """FixScaleCrop: shorter side to ``crop`` (bilinear image, nearest mask), then
    the centre ``crop`` x ``crop`` window."""
    Image = _pil()
    w, h = img.size
    if w > h:
        oh, ow = crop, int(1.0 * w * crop / h)
    else:
        ow, oh = crop, int(1.0 * h * crop / w)
    img = img.resize((ow, oh), Image.BILINEAR)
    mask = mask.resize((ow, oh), Image.NEAREST)
    x1 = int(round((ow - crop) / 2.0))
    y1 = int(round((oh - crop) / 2.0))
    box = (x1, y1, x1 + crop, y1 + crop)
    return img.crop(box), mask.crop(box)


def seg_normalize(img) -> np.ndarray:
    """The segmentation code's Normalize (custom_transforms.py:17-27) in its own
    numpy arithmetic: float32 image / 255 (fp32), then -= mean and /= std with the
    tuples as float64 arrays (computed in fp64, stored back to fp32) -- not
    torchvision's fp32 Normalize of the classification path."""
    x = np.array(img).astype(np.float32)
    x /= 255.0
    x -= MEAN
    x /= STD
    return x


def seg_transform(img, mask, crop: int):
    """The VOC validation transform (pascal.py:108-112): FixScaleCrop, Normalize,
    ToTensor.  Returns {"image": CHW float32, "label": HW float32} as the
    reference's ToTensor does (custom_transforms.py:33-46).  Pinned bit-exact to
    the reference (tests/golden/seg_transforms.npz)."""
    img, mask = fix_scale_crop(img, mask, crop)
    x = seg_normalize(img).transpose((2, 0, 1))
    m = np.array(mask).astype(np.float32)
    return {"image": torch.from_numpy(np.ascontiguousarray(x)).float(), "label": torch.from_numpy(m).float()}


class Evaluator:
    """Confusion-matrix segmentation metrics (labels outside [0, n) are ignored)."""

    def __init__(self, num_class: int):
        self.num_class = num_class
        self.confusion = np.zeros((num_class, num_class), dtype=np.int64)

    def add_batch(self, gt: np.ndarray, pred: np.ndarray):
        gt, pred = np.asarray(gt).ravel(), np.asarray(pred).ravel()
        keep = (gt >= 0) & (gt < self.num_class)   # float labels (the reference's ToTensor) too
        idx = self.num_class * gt[keep].astype(np.int64) + pred[keep].astype(np.int64)
        self.confusion += np.bincount(idx, minlength=self.num_class ** 2).reshape(self.num_class, self.num_class)

    def pixel_accuracy(self) -> float:
        return float(np.diag(self.confusion).sum() / max(self.confusion.sum(), 1))

    def mean_iou(self) -> float:
        c = self.confusion.astype(np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            iou = np.diag(c) / (c.sum(1) + c.sum(0) - np.diag(c))
        return float(np.nanmean(iou))


def forward_all(model, dataloader, device="cuda:0", num_class: int = 21) -> float:
    """Segmentation inference over the loader; returns the mean IoU."""
    ev = Evaluator(num_class)
    with torch.no_grad():
        for sample in dataloader:
            out = model(sample["image"].to(device))
            ev.add_batch(sample["label"].numpy(), out.argmax(1).cpu().numpy())
    return ev.mean_iou()


def inference_cls(model, root: str, device="cuda:0", batch_size: int = 256, workers: int = 4,
                  limit: Optional[int] = None) -> float:
    """Top-1 accuracy over an ImageFolder (main_dfq.py:91-113)."""
    ds = ImageFolder(root)
    if limit is not None:
        ds.samples = ds.samples[:limit]
    dl = torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=False, num_workers=workers,
                                     pin_memory=str(device).startswith("cuda"))
    correct = total = 0
    with torch.no_grad():
        for image, label in dl:
            pred = model(image.to(device)).argmax(1).cpu()
            correct += int((pred == label).sum())
            total += int(image.shape[0])
    return correct / max(total, 1)


def inference_seg(model, base_dir: str, device="cuda:0", batch_size: int = 32, workers: int = 2,
                  crop_size: int = 513) -> float:
    """mIoU over the VOC 2012 val split (main_dfq.py:80-89)."""
    ds = VOCSegmentation(crop_size, crop_size, base_dir=base_dir, split="val")
    dl = torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=False, num_workers=workers)
    return forward_all(model, dl, device, VOCSegmentation.NUM_CLASSES)


__all__: Sequence[str] = ["ImageFolder", "VOCSegmentation", "Evaluator", "cls_transform", "fix_scale_crop",
                          "seg_normalize", "seg_transform",
                          "forward_all", "inference_cls", "inference_seg"]
