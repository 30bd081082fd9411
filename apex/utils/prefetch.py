"""Input prefetcher with the fused K-09 normalize kernel.

Reference behaviour (examples/imagenet/main.py:241-273 ``data_prefetcher``): on a side
stream, copy the next uint8 batch to the GPU, cast to half, ``sub_(mean).div_(std)``; the
main stream waits on the side stream before consuming the batch. Here the cast + normalize
(+ NHWC->NCHW transpose when the loader yields HWC images) is one HIP kernel, the H2D copy is
from pinned memory, and ``record_stream`` keeps the caching allocator honest across streams.
"""
from __future__ import annotations

import torch

from .. import _ext

IMAGENET_MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
IMAGENET_STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)


def normalize_images(x, mean=IMAGENET_MEAN, std=IMAGENET_STD, nhwc=True, channels_last=False,
                     dtype=torch.float32):
    """uint8 images ([B,H,W,C] if ``nhwc`` else [B,C,H,W]) -> (x - mean) / std as ``dtype``
    in NCHW shape (channels_last memory format if requested)."""
    if _ext.use_native(x):
        return _ext.require().input_normalize(x, [float(m) for m in mean], [float(s) for s in std], nhwc,
                                              channels_last, dtype)
    xf = x.float()
    if nhwc:
        xf = xf.permute(0, 3, 1, 2)
    m = torch.tensor(mean, dtype=torch.float32, device=x.device).view(1, -1, 1, 1)
    s = torch.tensor(std, dtype=torch.float32, device=x.device).view(1, -1, 1, 1)
    y = ((xf - m) / s).to(dtype)
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    return y.contiguous(memory_format=fmt)


class DataPrefetcher:
    """Iterates ``loader`` (yielding (uint8 images, targets)) one batch ahead on a side stream."""

    def __init__(self, loader, device=None, mean=IMAGENET_MEAN, std=IMAGENET_STD, nhwc=True,
                 channels_last=False, dtype=torch.float32):
        self.loader = iter(loader)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.kw = dict(mean=mean, std=std, nhwc=nhwc, channels_last=channels_last, dtype=dtype)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self._preload()

    def _preload(self):
        try:
            x, y = next(self.loader)
        except StopIteration:
            self.next_input = self.next_target = None
            return
        if not self.cuda:
            self.next_input = normalize_images(x, **self.kw)
            self.next_target = y
            return
        with torch.cuda.stream(self.stream):
            xg = x.pin_memory().to(self.device, non_blocking=True) if not x.is_cuda else x
            self.next_target = y.to(self.device, non_blocking=True)
            self.next_input = normalize_images(xg, **self.kw)

    def next(self):
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        x, y = self.next_input, self.next_target
        if self.cuda and x is not None:
            x.record_stream(torch.cuda.current_stream(self.device))
            y.record_stream(torch.cuda.current_stream(self.device))
        self._preload()
        return x, y

    def __iter__(self):
        while True:
            x, y = self.next()
            if x is None:
                return
            yield x, y
