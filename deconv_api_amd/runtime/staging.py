"""Pinned host staging ring + copy/compute/copy-back streams for request batches.

The reference decodes, resizes and runs every request serially on the event loop
(app/main.py:46-78). Here one batch of decoded images of ANY sizes becomes:

  host   pack the images back to back into one pinned slot (+ a {offset, H, W, mode} table)
  copy   ONE H2D copy of the slot on the copy stream                       (event h2d)
  comp   ONE resize(+preprocess) launch for the whole batch (csrc/misc.hip:resize_batch_kernel),
         then the engine, on the compute stream                            (event comp)
  back   D2D of the mosaics into the slot's device buffer (the graph-owned output is free for
         the next replay at once), D2H into a pinned block on the copy-back stream

Slots rotate (``slots`` deep), so batch i+1's upload and resize overlap batch i's engine work
and batch i-1's copy-back; a slot is reused only after its previous batch's events completed.
Per-stage hipEvent timings are exported as Prometheus histograms (utils/metrics.py).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ..ops import native
from ..ops.misc import resize_mode
from ..utils import metrics as M


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class Staged:
    """One in-flight batch: events and buffers of its slot."""
    slot: int
    n: int
    ev_h2d0: torch.cuda.Event
    ev_h2d1: torch.cuda.Event
    ev_comp0: torch.cuda.Event
    ev_comp1: Optional[torch.cuda.Event] = None
    ev_back1: Optional[torch.cuda.Event] = None
    host_out: Optional[torch.Tensor] = None
    scans: Optional[torch.Tensor] = None  # GPU JPEG: the device scans (copied once their size is known)
    hw: tuple = (0, 0)


@dataclass
class GpuScans:
    """A batch's responses as GPU-encoded JPEG scans on the host (codec.gpu_data_urls input)."""
    packed: torch.Tensor  # uint8 [off[-1]]
    off: torch.Tensor     # int64 [n + 1]
    H: int
    W: int

    def __len__(self) -> int:
        return self.off.numel() - 1


def resize_batch(images: List[np.ndarray], out: torch.Tensor) -> torch.Tensor:
    """Unstaged one-shot form (tools / tests): pack, upload synchronously, one batched resize."""
    offs, end = [], 0
    for im in images:
        offs.append(end)
        end = _round_up(end + im.size, 16)
    blob = np.zeros(max(end, 16), np.uint8)
    tab = np.zeros((len(images), 4), np.int64)
    for b, (im, o) in enumerate(zip(images, offs)):
        blob[o:o + im.size] = np.ascontiguousarray(im).reshape(-1)
        tab[b] = (o, im.shape[0], im.shape[1], resize_mode(im.shape[0], im.shape[1], out.shape[1], out.shape[2]))
    native.lib().resize_batch(torch.from_numpy(blob).to(out.device), torch.from_numpy(tab).to(out.device),
                              out[: len(images)], end)
    return out


class StagingRing:
    def __init__(self, device: torch.device, slots: int = 3, slot_bytes: int = 32 << 20, max_images: int = 256):
        assert device.type == "cuda"
        self.device = device
        self.slots = slots
        self.max_images = max_images
        from .streams import independent_stream

        # upload / copy-back streams on hardware queues apart from the compute stream's (streams.py)
        self.compute_stream = torch.cuda.Stream(device)
        self.copy_stream = independent_stream(device, [self.compute_stream])
        self.back_stream = independent_stream(device, [self.compute_stream, self.copy_stream])
        self._bytes = [0] * slots
        self.host: List[Optional[torch.Tensor]] = [None] * slots
        self.dev: List[Optional[torch.Tensor]] = [None] * slots
        self.tab_host = torch.empty(slots, max_images, 4, dtype=torch.int64, pin_memory=True)
        self.tab_dev = torch.empty(slots, max_images, 4, dtype=torch.int64, device=device)
        self.out_dev: List[Optional[torch.Tensor]] = [None] * slots
        self.busy: List[Optional[Staged]] = [None] * slots  # the batch last staged in each slot
        # per slot: recorded on the compute stream right after the slot's resize launch, the last
        # reader of its device blob and table; the next upload into the slot waits for that only
        self.resized: List[Optional[torch.cuda.Event]] = [None] * slots
        self._next = 0
        self._lock = threading.Lock()
        for i in range(slots):
            self._ensure(i, slot_bytes)

    def _ensure(self, i: int, nbytes: int) -> None:
        if self._bytes[i] >= nbytes:
            return
        cap = 1 << max(20, (nbytes - 1).bit_length())
        self.host[i] = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
        self.dev[i] = torch.empty(cap, dtype=torch.uint8, device=self.device)
        self._bytes[i] = cap

    def _acquire(self) -> int:
        with self._lock:
            i = self._next
            self._next = (i + 1) % self.slots
        prev = self.busy[i]
        if prev is not None:  # the slot's previous batch must be fully done with its buffers
            (prev.ev_back1 or prev.ev_comp1 or prev.ev_h2d1).synchronize()
        return i

    # ------------------------------------------------------------------ upload + resize
    def stage(self, images: List[np.ndarray], out: torch.Tensor) -> Staged:
        """Pack ``images`` (uint8 HxWx3, any sizes) into a slot, upload, and resize into ``out``
        ([n, S, S, Cpad] bf16 preprocessed, or [n, S, S, 3] uint8) on the compute stream."""
        n = len(images)
        assert 0 < n <= self.max_images and out.shape[0] >= n
        S_h, S_w = out.shape[1], out.shape[2]
        i = self._acquire()
        offs, end = [], 0
        for im in images:
            assert im.dtype == np.uint8 and im.ndim == 3 and im.shape[2] == 3
            offs.append(end)
            end = _round_up(end + im.size, 16)
        self._ensure(i, end)
        hv = self.host[i].numpy()
        tab = self.tab_host[i].numpy()
        for b, (im, o) in enumerate(zip(images, offs)):
            hv[o:o + im.size] = np.ascontiguousarray(im).reshape(-1)
            tab[b] = (o, im.shape[0], im.shape[1], resize_mode(im.shape[0], im.shape[1], S_h, S_w))
        st = Staged(i, n, torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
                    torch.cuda.Event(enable_timing=True))
        cur = torch.cuda.current_stream(self.device)
        if self.resized[i] is not None:
            # the slot's previous resize must have read its blob; NOT wait_stream(cur), which would
            # also wait for the previous batch's engine work and serialize upload behind compute
            self.copy_stream.wait_event(self.resized[i])
        with torch.cuda.stream(self.copy_stream):
            st.ev_h2d0.record()
            self.dev[i][:end].copy_(self.host[i][:end], non_blocking=True)
            self.tab_dev[i, :n].copy_(self.tab_host[i, :n], non_blocking=True)
            st.ev_h2d1.record()
        cur.wait_event(st.ev_h2d1)
        st.ev_comp0.record(cur)
        native.lib().resize_batch(self.dev[i], self.tab_dev[i, :n], out[:n], end)
        ev = torch.cuda.Event()
        ev.record(cur)
        self.resized[i] = ev
        self.busy[i] = st
        return st

    # ------------------------------------------------------------------ copy back
    def copy_back(self, st: Staged, mosaic: torch.Tensor) -> Staged:
        """Enqueue D2D (into the slot's device buffer) + D2H (into its pinned output) of the
        first ``st.n`` rows of ``mosaic``; the caller's stream may reuse ``mosaic`` right after."""
        n = st.n
        i = st.slot
        shape = (self.max_images, *mosaic.shape[1:])
        if self.out_dev[i] is None or tuple(self.out_dev[i].shape[1:]) != tuple(mosaic.shape[1:]):
            self.out_dev[i] = torch.empty(shape, dtype=mosaic.dtype, device=self.device)
        # the host side is a per-batch pinned block from torch's caching host allocator: the
        # completion thread may still be reading batch i's result when batch i + slots copies back
        host = torch.empty((n, *mosaic.shape[1:]), dtype=mosaic.dtype, pin_memory=True)
        cur = torch.cuda.current_stream(self.device)
        self.out_dev[i][:n].copy_(mosaic[:n])
        st.ev_comp1 = torch.cuda.Event(enable_timing=True)
        st.ev_comp1.record(cur)
        self.back_stream.wait_event(st.ev_comp1)
        with torch.cuda.stream(self.back_stream):
            host.copy_(self.out_dev[i][:n], non_blocking=True)
            st.ev_back1 = torch.cuda.Event(enable_timing=True)
            st.ev_back1.record()
        st.host_out = host
        return st

    def copy_back_jpeg(self, st: Staged, mosaic: torch.Tensor, quality: int) -> Staged:
        """GPU JPEG instead of raw mosaics: the first ``st.n`` mosaics are encoded on the compute
        stream (csrc/jpeg_gpu.hip) and only the scan offsets are copied back here; ``finish``
        copies the scans (~10x fewer bytes than the mosaics) once their total size is known."""
        from ..codec.image import encode_gpu

        n = st.n
        cur = torch.cuda.current_stream(self.device)
        packed, off = encode_gpu(mosaic[:n], quality)
        st.ev_comp1 = torch.cuda.Event(enable_timing=True)
        st.ev_comp1.record(cur)
        host_off = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
        self.back_stream.wait_event(st.ev_comp1)
        # both device blocks are read on back_stream after this function returns: without
        # record_stream the compute stream's pool could hand `off` to the next batch before the
        # D2H below ran (corrupt scan offsets)
        packed.record_stream(self.back_stream)
        off.record_stream(self.back_stream)
        with torch.cuda.stream(self.back_stream):
            host_off.copy_(off, non_blocking=True)
            st.ev_back1 = torch.cuda.Event(enable_timing=True)
            st.ev_back1.record()
        st.host_out, st.scans, st.hw = host_off, packed, (mosaic.shape[1], mosaic.shape[2])
        return st

    def finish(self, st: Staged):
        """Wait for the batch's copy-back; record per-stage timings; return a host copy (the
        mosaics, or GpuScans for a copy_back_jpeg batch)."""
        st.ev_back1.synchronize()
        M.STAGE_TIME.observe(st.ev_h2d0.elapsed_time(st.ev_h2d1) / 1e3, stage="h2d")
        M.STAGE_TIME.observe(st.ev_comp0.elapsed_time(st.ev_comp1) / 1e3, stage="compute")
        M.STAGE_TIME.observe(st.ev_comp1.elapsed_time(st.ev_back1) / 1e3, stage="d2h")
        if st.scans is not None:
            total = int(st.host_out[-1])
            packed = torch.empty(total, dtype=torch.uint8, pin_memory=True)
            with torch.cuda.stream(self.back_stream):
                packed.copy_(st.scans[:total], non_blocking=True)
            self.back_stream.synchronize()
            st.scans = None
            return GpuScans(packed, st.host_out, *st.hw)
        return st.host_out.numpy()
