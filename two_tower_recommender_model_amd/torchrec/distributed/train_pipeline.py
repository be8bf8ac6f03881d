"""torchrec.distributed.TrainPipelineSparseDist on HIP streams.

``TrainPipelineSparseDist(model, optimizer, device)`` and ``progress(iterator)`` as driven by the
reference's train/evaluate loops (03_model_training.py:545, :618, :648): each call trains (or, in
``eval()`` mode, only runs forward on) one batch and returns the model output's second element
``(loss, logits, labels)``; it raises StopIteration once the iterator is drained.

Three stages over three streams, as torchrec's pipeline:
  memcpy stream     host -> device copy of batch i+2
  data-dist stream  input_dist of batch i+1 in every ShardedEmbeddingBagCollection of the model
                    (KJT permute / bucketize + the counts, lengths and ids all-to-alls)
  current stream    forward / backward / optimizer.step of batch i (its lookups consume the staged
                    input_dist: ``ShardedEmbeddingBagCollection.prefetch``)
Batch i's kernels are queued before batch i+1's input_dist starts, so the host-side waits of that
input_dist (its split sizes) overlap batch i's device work. input_dist reads only ids, so running it
before batch i's table update is exact. Without sharded modules the pipeline has two stages.

Training ``progress`` on the reference's two-tower model (single-hot KJTs, bf16 towers) is
dispatched to the fused steps (``two_tower_recommender_model_amd.dropin``) on the model's own
storage: at world size 1 the production ring (three fused launches per batch replayed as HIP
graphs), at world size W > 1 the pipelined sharded step on the DMP plan's shards (two fixed-size
RCCL all-to-alls per batch inside the HIP graphs).
``_fused_reason`` says why a pipeline did not dispatch; ``TT_DROPIN_FUSED=0`` turns it off.
"""
from __future__ import annotations

from typing import Any, Iterator, List, Optional

import torch


class _Staged:
    __slots__ = ("batch", "h2d", "dist")

    def __init__(self, batch, h2d):
        self.batch = batch
        self.h2d = h2d
        self.dist = False


class TrainPipelineBase:
    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, device: torch.device):
        self._model = model
        self._optimizer = optimizer
        self._device = torch.device(device)
        self._cuda = self._device.type == "cuda"
        self._memcpy_stream = torch.cuda.Stream(device=self._device) if self._cuda else None
        self._cur: Optional[_Staged] = None    # batch i (input_dist staged)
        self._next: Optional[_Staged] = None   # batch i+1 (copy issued)
        self._connected = False
        self._fused = None          # dropin.FusedDropin once built (False: not applicable)
        self._fused_reason = "not tried"
        self._pushback: List[Any] = []

    def _sharded(self) -> List[Any]:
        return []

    def _fetch(self, it: Iterator) -> Optional[_Staged]:
        if self._pushback:  # batches a fused drop-in fetched ahead and handed back (dropin.drain_to)
            batch = self._pushback.pop(0)
        else:
            try:
                batch = next(it)
            except StopIteration:
                return None
        if not self._cuda:
            return _Staged(batch.to(self._device, non_blocking=True), None)
        with torch.cuda.stream(self._memcpy_stream):
            b = batch.to(self._device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._memcpy_stream)
        return _Staged(b, ev)

    def _start_sparse_data_dist(self, st: Optional[_Staged]) -> None:
        pass

    def _wait(self, st: _Staged) -> None:
        if st.h2d is not None:
            cur = torch.cuda.current_stream(self._device)
            cur.wait_event(st.h2d)
            if hasattr(st.batch, "record_stream"):
                st.batch.record_stream(cur)

    def progress(self, dataloader_iter: Iterator) -> Any:
        if self._model.training and self._cur is None:
            if self._fused is None:
                from ...dropin import FusedDropin

                fd, self._fused_reason = FusedDropin.build(self)
                self._fused = fd if fd is not None else False
            if self._fused:
                return self._fused.progress(dataloader_iter)
        elif self._fused and self._fused.pending():
            self._fused.drain_to(self)  # eval mid-chunk: the staged batches go the generic way
        if self._cur is None:
            # (re)fill: batch i copied and its input_dist staged, batch i+1's copy issued
            self._cur = self._fetch(dataloader_iter)
            if self._cur is None:
                raise StopIteration
            self._start_sparse_data_dist(self._cur)
            self._next = self._fetch(dataloader_iter)
        st = self._cur
        self._wait(st)
        training = self._model.training
        if training:
            self._optimizer.zero_grad(set_to_none=True)
        losses, output = self._model(st.batch)
        if training:
            torch.sum(losses, dim=0).backward()
            self._optimizer.step()
        # stages 2 and 1 for the following batches, behind batch i's queued kernels
        self._cur, self._next = self._next, None
        if self._cur is not None:
            self._start_sparse_data_dist(self._cur)
            self._next = self._fetch(dataloader_iter)
        return output


class TrainPipelineSparseDist(TrainPipelineBase):
    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, device: torch.device,
                 execute_all_batches: bool = True, apply_jit: bool = False):
        super().__init__(model, optimizer, device)
        self._data_dist_stream = torch.cuda.Stream(device=self._device) if self._cuda else None

    def _sharded(self) -> List[Any]:
        from .embeddingbag import ShardedEmbeddingBagCollection

        return [m for m in self._model.modules() if isinstance(m, ShardedEmbeddingBagCollection)]

    def _start_sparse_data_dist(self, st: Optional[_Staged]) -> None:
        mods = self._sharded()
        if st is None or st.dist or not mods:
            return
        kjt = getattr(st.batch, "sparse_features", None)
        if kjt is None:
            return
        # only modules the batch KJT feeds whole (torchrec traces which module receives the input;
        # a module fed a derived KJT runs its own input_dist in forward)
        mods = [m for m in mods if m.accepts(kjt)]
        if self._data_dist_stream is None:
            for m in mods:
                m.prefetch(kjt)
        else:
            with torch.cuda.stream(self._data_dist_stream):
                if st.h2d is not None:
                    self._data_dist_stream.wait_event(st.h2d)
                for m in mods:
                    m.prefetch(kjt)
        st.dist = True
