"""``DriveDataset`` (my_dataset.py:15-257) feeding the device augmentation.

Same constructor, directory scan and sample order as the reference: ``root/seg/
{training,val,test}/images/<patient>/<sequence>/<slice>.{jpg,png}`` with the label at
``labels/<patient>/<first sequence>/<slice>.{png,jpg}``, sequences ``VIBRANT+C1..8``
(or ``SUB1..8`` with ``use_subtraction``), PK maps ``pk_maps/<patient>/{ktrans,ve,
vp}.png`` with ``use_pk_maps``.

With ``transforms`` a :class:`stfunet.augment.DeviceAugment`, ``__getitem__`` returns
the decoded uint8 frames [F][H][W] (T frames, then the PK maps), the 0/1 uint8 mask and
the sample's drawn parameters -- the draws happen in the worker, in the reference's
order -- and ``collate_fn`` (still in the worker) builds the batch's augmentation plan
(one byte blob).  :class:`DeviceLoader` copies each plan to the GPU and runs the
kernels: the workers do file decoding only, the geometry runs on the device.  With
``transforms=None`` the reference's no-transform branch is kept (fp32 /255 tensors,
int64 mask; my_dataset.py:219-232) and ``collate_fn`` stacks as the reference does
(targets padded with 255, ``cat_list``).

Decoding: Pillow ``convert('L')`` where the reference uses ``cv2.imread(...,
IMREAD_GRAYSCALE)`` (cv2 is absent from this image): identical for 8-bit grayscale
PNGs; for JPEG or colour files the two decoders / luma rules can differ by one level
(unpinned).  A missing PK map reads as zeros, as in the reference (:226-228).
"""
import os

import numpy as np
import torch
from torch.utils.data import Dataset

from .augment import DeviceAugment


def _read_gray(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.array(im.convert("L"))


class DriveDataset(Dataset):
    def __init__(self, root, mode, transforms=None, sequence_types=None, use_subtraction=False,
                 use_pk_maps=False):
        super().__init__()
        assert mode in ("train", "val", "test"), f"unsupported mode: {mode}"
        self.mode = mode
        self.flag = {"train": "training", "val": "val", "test": "test"}[mode]
        self.use_pk_maps = use_pk_maps
        if sequence_types is None:
            sequence_types = [f"SUB{i}" for i in range(1, 9)] if use_subtraction else \
                [f"VIBRANT+C{i}" for i in range(1, 9)]
        self.sequence_types = sequence_types
        data_root = os.path.join(root, "seg", self.flag)
        assert os.path.exists(data_root), f"path '{data_root}' does not exists."
        self.transforms = transforms
        if transforms is not None and not isinstance(transforms, DeviceAugment):
            raise TypeError("transforms must be a stfunet.augment.DeviceAugment or None")
        img_dir, mask_dir = os.path.join(data_root, "images"), os.path.join(data_root, "labels")
        assert os.path.exists(img_dir), f"path '{img_dir}' does not exists."
        assert os.path.exists(mask_dir), f"path '{mask_dir}' does not exists."
        self.patient_data = []
        for patient in os.listdir(img_dir):                    # reference order (unsorted listdir)
            pimg, pmask = os.path.join(img_dir, patient), os.path.join(mask_dir, patient)
            if not os.path.isdir(pimg) or not os.path.isdir(pmask):
                continue
            if not all(os.path.exists(os.path.join(pimg, s)) for s in self.sequence_types):
                continue
            pk_path = None
            if use_pk_maps:
                pk_path = os.path.join(data_root, "pk_maps", patient)
                if not os.path.exists(pk_path):
                    continue
            first = os.path.join(pimg, self.sequence_types[0])
            for img_file in [f for f in os.listdir(first) if f.endswith(".jpg") or f.endswith(".png")]:
                paths = [os.path.join(pimg, s, img_file) for s in self.sequence_types]
                if not all(os.path.exists(p) for p in paths):
                    continue
                base = os.path.splitext(img_file)[0]
                mask_path = None
                for name in (f"{base}.png", f"{base}.jpg"):
                    cand = os.path.join(pmask, self.sequence_types[0], name)
                    if os.path.exists(cand):
                        mask_path = cand
                        break
                if mask_path is None:
                    continue
                self.patient_data.append({"patient_id": patient, "image_paths": paths, "mask_path": mask_path,
                                          "pk_maps_path": pk_path})

    def __len__(self):
        return len(self.patient_data)

    def _raw(self, idx):
        item = self.patient_data[idx]
        frames = [_read_gray(p) for p in item["image_paths"]]
        mask = (_read_gray(item["mask_path"]) / 255).astype(np.uint8)         # :201-204
        if self.use_pk_maps:
            for name in ("ktrans", "ve", "vp"):
                p = os.path.join(item["pk_maps_path"], f"{name}.png")
                frames.append(_read_gray(p) if os.path.exists(p) else np.zeros_like(frames[0]))
        return np.stack(frames), mask

    def __getitem__(self, idx):
        frames, mask = self._raw(idx)
        if self.transforms is not None:
            F, H, W = frames.shape
            return frames, mask, self.transforms.draw_sample(F, H, W)
        x = torch.from_numpy(frames).float().div(255.0).unsqueeze(1)             # [F][1][H][W]
        return x, torch.from_numpy(mask).long()

    def collate_fn(self, batch):
        """Device-augmentation batches -> the augmentation plan (numpy, in the worker);
        tensor batches -> the reference's stack + ``cat_list(targets, 255)``."""
        if self.transforms is not None:
            frames, masks, params = zip(*batch)
            return self.transforms.plan(list(frames), list(masks), list(params))
        xs, ts = zip(*batch)
        return torch.stack(xs), cat_list(ts, fill_value=255)


def cat_list(images, fill_value=0):
    """my_dataset.py:262-272."""
    if len(images) == 0:
        return torch.zeros((0,))
    max_size = tuple(max(s) for s in zip(*[img.shape for img in images]))
    out = images[0].new(*((len(images),) + max_size)).fill_(fill_value)
    for img, pad in zip(images, out):
        pad[..., :img.shape[-2], :img.shape[-1]].copy_(img)
    return out


class DeviceLoader:
    """Iterate a DataLoader over a device-augmented ``DriveDataset``: each worker-built
    plan is copied to the GPU (one pinned copy) and augmented there; yields
    (x fp32 [B][F][1][h][w], target int64 [B][h][w]) on the device, the layout the
    reference's loader yields (my_dataset.py:242-257)."""

    def __init__(self, loader, augment):
        self.loader, self.augment = loader, augment

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for plan in self.loader:
            yield self.augment.launch(self.augment.to_device(plan))
