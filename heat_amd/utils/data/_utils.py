"""
Dataset-preparation utilities (reference ``heat/utils/data/_utils.py``): index files for NVIDIA
DALI TFRecord readers and the merge of ImageNet TFRecord shards into HDF5 files for
:class:`~heat_amd.utils.data.partial_dataset.PartialH5Dataset`.

Both are offline tools with optional dependencies (``tfrecord2idx`` from DALI, TensorFlow for
decoding records, ``h5py``); they raise ``ImportError`` naming what is missing.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import Optional

__all__ = ["dali_tfrecord2idx", "merge_files_imagenet_tfrecord"]


def dali_tfrecord2idx(train_dir: str, train_idx_dir: str, val_dir: str, val_idx_dir: str) -> None:
    """Create the DALI index file of every TFRecord shard in ``train_dir`` / ``val_dir`` (run the
    ``tfrecord2idx`` tool shipped with DALI once per file)."""
    tool = shutil.which("tfrecord2idx")
    if tool is None:
        raise ImportError("dali_tfrecord2idx needs NVIDIA DALI's 'tfrecord2idx' executable on PATH")
    for src, dst in ((train_dir, train_idx_dir), (val_dir, val_idx_dir)):
        os.makedirs(dst, exist_ok=True)
        for name in sorted(os.listdir(src)):
            out = os.path.join(dst, name + ".idx")
            if not os.path.exists(out):
                subprocess.run([tool, os.path.join(src, name), out], check=True)


def merge_files_imagenet_tfrecord(folder_name: str, output_folder: Optional[str] = None) -> None:
    """Merge the ImageNet TFRecord shards of ``folder_name`` into ``imagenet_merged.h5`` /
    ``imagenet_merged_validation.h5`` (JPEG bytes as variable-length uint8 rows, labels, file
    names), the layout PartialH5Dataset streams."""
    try:
        import h5py
        import numpy as np
        import tensorflow as tf  # noqa: F401  (record parsing)
    except ImportError as e:
        raise ImportError("merge_files_imagenet_tfrecord needs h5py and tensorflow: {}".format(e)) from e
    output_folder = output_folder or folder_name
    feature = {"image/encoded": tf.io.FixedLenFeature([], tf.string),
               "image/class/label": tf.io.FixedLenFeature([], tf.int64),
               "image/filename": tf.io.FixedLenFeature([], tf.string)}
    for kind, prefix in (("", "train"), ("_validation", "validation")):
        files = sorted(os.path.join(folder_name, f) for f in os.listdir(folder_name) if f.startswith(prefix))
        if not files:
            continue
        with h5py.File(os.path.join(output_folder, "imagenet_merged{}.h5".format(kind)), "w") as out:
            vlen = h5py.vlen_dtype(np.dtype("uint8"))
            imgs = out.create_dataset("images", (0,), maxshape=(None,), dtype=vlen, chunks=True)
            labels = out.create_dataset("metadata", (0,), maxshape=(None,), dtype="i8", chunks=True)
            names = out.create_dataset("file_info", (0,), maxshape=(None,), dtype=h5py.string_dtype(),
                                       chunks=True)
            n = 0
            for rec in tf.data.TFRecordDataset(files):
                ex = tf.io.parse_single_example(rec, feature)
                for ds in (imgs, labels, names):
                    ds.resize((n + 1,))
                imgs[n] = np.frombuffer(ex["image/encoded"].numpy(), dtype=np.uint8)
                labels[n] = int(ex["image/class/label"].numpy())
                names[n] = ex["image/filename"].numpy().decode()
                n += 1
