"""torchrec.distributed.TrainPipelineSparseDist on HIP streams.

``TrainPipelineSparseDist(model, optimizer, device)`` and ``progress(iterator)`` as driven by the
reference's train/evaluate loops (03_model_training.py:545, :618, :648): each call trains (or, in
``eval()`` mode, only runs forward on) one batch and returns the model output's second element
``(loss, logits, labels)``; it raises StopIteration once the iterator is drained. The next batch's
host->device copy is issued on a separate copy stream while the current batch computes (the
H2D stage of torchrec's 3-stage pipeline; input_dist runs inside the sharded module's forward).
"""
from __future__ import annotations

from typing import Any, Iterator, Optional

import torch


class TrainPipelineBase:
    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, device: torch.device):
        self._model = model
        self._optimizer = optimizer
        self._device = torch.device(device)
        self._cur: Optional[Any] = None
        self._next: Optional[Any] = None
        self._next_event = None
        self._connected = False
        self._memcpy_stream = torch.cuda.Stream(device=self._device) if self._device.type == "cuda" else None

    def _to_device(self, batch):
        if self._memcpy_stream is None:
            return batch.to(self._device, non_blocking=True), None
        with torch.cuda.stream(self._memcpy_stream):
            b = batch.to(self._device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._memcpy_stream)
        return b, ev

    def _fetch(self, it: Iterator):
        batch = next(it)  # StopIteration propagates
        return self._to_device(batch)

    def progress(self, dataloader_iter: Iterator) -> Any:
        if self._cur is None:
            if self._next is not None:
                self._cur, ev = self._next, self._next_event
                self._next = self._next_event = None
            else:
                self._cur, ev = self._fetch(dataloader_iter)
            if ev is not None:
                torch.cuda.current_stream(self._device).wait_event(ev)
                if hasattr(self._cur, "record_stream"):
                    self._cur.record_stream(torch.cuda.current_stream(self._device))
        batch = self._cur
        # stage the next batch's copy while this one computes
        if self._next is None:
            try:
                self._next, self._next_event = self._fetch(dataloader_iter)
            except StopIteration:
                self._next = self._next_event = None
        training = self._model.training
        if training:
            self._optimizer.zero_grad(set_to_none=True)
        losses, output = self._model(batch)
        if training:
            torch.sum(losses, dim=0).backward()
            self._optimizer.step()
        self._cur = None
        return output


class TrainPipelineSparseDist(TrainPipelineBase):
    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, device: torch.device,
                 execute_all_batches: bool = True, apply_jit: bool = False):
        super().__init__(model, optimizer, device)
