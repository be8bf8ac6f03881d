"""torchrec.modules.mlp.MLP / Perceptron on the bf16-MFMA tower GEMMs.

``MLP(in_size, layer_sizes, device)`` (03_model_training.py:411-412) = Sequential of Perceptrons,
each ``relu(Linear(x))`` — ReLU on EVERY layer including the last (torchrec semantics), parameters
at ``_mlp[i]._linear.{weight,bias}`` (03:1143). Each Perceptron is one fused HIP launch forward
(GEMM + bias + ReLU epilogue) and two backward (dX with the ReLU mask fused into the operand load;
dW/db split-K with a fixed-order reduction). fp32 master weights, bf16 MFMA, fp32 accumulate.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Union

import torch
from torch import nn

from ... import _lib, ops


#: default compute mode of new Perceptrons: "bf16" (bf16 MFMA operands, the production mode named
#: by the north star) or "fp32" (exact fp32 MFMA operands, parity with the reference's fp32 MLP)
TOWER_PRECISION = "bf16"


class _LinearReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, precision):
        if x.stride(-1) != 1:
            x = x.contiguous()
        (y,) = ops.linear_fwd([x], [weight.detach()], [bias.detach() if bias is not None else None], relu=True,
                              precision=precision)
        ctx.save_for_backward(x, weight, y)
        ctx.has_bias = bias is not None
        ctx.precision = precision
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            (dx,) = ops.linear_bwd_data([dy], [y], [weight.detach()], relu=True, precision=ctx.precision)
        dw = db = None
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            (dw,), (db,) = ops.linear_bwd_weight([dy], [y], [x], relu=True, precision=ctx.precision)
        return dx, dw, (db if ctx.has_bias else None), None


def _is_relu(act) -> bool:
    return act is torch.relu or act is torch.nn.functional.relu or isinstance(act, nn.ReLU) or act == "relu"


class Perceptron(nn.Module):
    def __init__(self, in_size: int, out_size: int, bias: bool = True,
                 activation: Union[nn.Module, Callable[[torch.Tensor], torch.Tensor]] = torch.relu,
                 device: Optional[torch.device] = None, dtype: torch.dtype = torch.float32):
        super().__init__()
        if not _is_relu(activation):
            raise NotImplementedError("the MI355X Perceptron fuses ReLU (the torchrec default); other activations "
                                      "are not on the reference's path")
        self._out_size = out_size
        self._in_size = in_size
        self._linear = nn.Linear(in_size, out_size, bias=bias, device=device, dtype=dtype)
        self._activation_fn = activation
        self.precision = TOWER_PRECISION

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            raise _lib.TTError("Perceptron runs on the MI355X kernels only: move the model/input to the GPU")
        return _LinearReLU.apply(x, self._linear.weight, self._linear.bias, self.precision)


class MLP(nn.Module):
    def __init__(self, in_size: int, layer_sizes: List[int], bias: bool = True,
                 activation: Union[str, Callable[[], nn.Module], nn.Module, Callable[[torch.Tensor], torch.Tensor]] = torch.relu,
                 device: Optional[torch.device] = None, dtype: torch.dtype = torch.float32):
        super().__init__()
        if activation == "relu":
            activation = torch.relu
        self._mlp = nn.Sequential(*[
            Perceptron(layer_sizes[i - 1] if i > 0 else in_size, layer_sizes[i], bias=bias, activation=activation,
                       device=device, dtype=dtype)
            for i in range(len(layer_sizes))
        ])

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        return self._mlp(input)
