"""``paddle.static.nn`` — layer-building functions for static Programs.

Parity: reference `python/paddle/static/nn/__init__.py` / `static/nn/common.py:fc` and
`fluid/layers/nn.py` (conv2d, batch_norm, layer_norm, embedding, prelu, group_norm,
instance_norm, create_parameter, cond). Parameters are created eagerly as real tensors (the
reference's startup-program initialisers) and registered as persistable Program variables the
first time an op consumes them; the ops themselves are recorded into the current Program.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import nn as _nn
from ..nn import functional as F
from .framework import Variable, _record


def _act(x, act):
    if not act:
        return x
    return getattr(F, act)(x)


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    xs = x if isinstance(x, (list, tuple)) else [x]
    outs = []
    for xi in xs:
        in_dim = int(np.prod(xi.shape[num_flatten_dims:]))
        lin = _nn.Linear(in_dim, size, weight_attr=weight_attr, bias_attr=bias_attr if len(outs) == 0 else False)
        if xi.dim() != num_flatten_dims + 1:
            xi = xi.reshape(list(xi.shape[:num_flatten_dims]) + [in_dim])
        outs.append(lin(xi))
    out = outs[0]
    for o in outs[1:]:
        out = out + o
    return _act(out, activation)


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,  # noqa: A002
           param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCHW"):
    conv = _nn.Conv2D(input.shape[1], num_filters, filter_size, stride, padding, dilation, groups or 1,
                      weight_attr=param_attr, bias_attr=bias_attr)
    return _act(conv(input), act)


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1,  # noqa: A002
                     dilation=1, groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None,
                     name=None, data_format="NCHW"):
    conv = _nn.Conv2DTranspose(input.shape[1], num_filters, filter_size, stride, padding,
                               groups=groups or 1, dilation=dilation, weight_attr=param_attr,
                               bias_attr=bias_attr)
    return _act(conv(input), act)


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-5, param_attr=None,  # noqa: A002
               bias_attr=None, data_layout="NCHW", in_place=False, name=None, moving_mean_name=None,
               moving_variance_name=None, do_model_average_for_mean_and_var=True,
               use_global_stats=False):
    bn = _nn.BatchNorm2D(input.shape[1], momentum, epsilon, param_attr, bias_attr) if input.dim() == 4 \
        else _nn.BatchNorm1D(input.shape[1], momentum, epsilon, param_attr, bias_attr)
    if is_test or use_global_stats:
        bn.eval()
    return _act(bn(input), act)


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-5, param_attr=None,  # noqa: A002
               bias_attr=None, act=None, name=None):
    shape = list(input.shape[begin_norm_axis:])
    ln = _nn.LayerNorm(shape, epsilon, param_attr if scale else False, bias_attr if shift else False)
    return _act(ln(input), act)


def group_norm(input, groups, epsilon=1e-5, param_attr=None, bias_attr=None, act=None,  # noqa: A002
               data_layout="NCHW", name=None):
    gn = _nn.GroupNorm(groups, input.shape[1], epsilon, param_attr, bias_attr)
    return _act(gn(input), act)


def instance_norm(input, epsilon=1e-5, param_attr=None, bias_attr=None, name=None):  # noqa: A002
    return _nn.InstanceNorm2D(input.shape[1], epsilon, weight_attr=param_attr, bias_attr=bias_attr)(input)


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None,  # noqa: A002
              param_attr=None, dtype="float32"):
    emb = _nn.Embedding(size[0], size[1], padding_idx, sparse=is_sparse, weight_attr=param_attr)
    return emb(input)


sparse_embedding = embedding


def prelu(x, mode="all", param_attr=None, data_format="NCHW", name=None):
    n = 1 if mode == "all" else x.shape[1]
    return _nn.PReLU(n, weight_attr=param_attr)(x)


def create_parameter(shape, dtype="float32", name=None, attr=None, is_bias=False, default_initializer=None):
    from ..nn.layer.base import Layer
    return Layer().create_parameter(shape, attr, dtype, is_bias, default_initializer)


def cond(pred, true_fn=None, false_fn=None, name=None, return_names=None):
    """Reference `layers/control_flow.py` cond: a Python bool / concrete tensor picks a branch
    eagerly; a Program Variable records a ``cond`` op with one sub-block per branch
    (`control_flow.py`) and the Executor runs only the branch the predicate selects."""
    if not isinstance(pred, Variable):
        p = bool(pred.reshape(-1)[0]) if isinstance(pred, torch.Tensor) else bool(pred)
        return (true_fn() if true_fn else None) if p else (false_fn() if false_fn else None)
    from .control_flow import cond as _cond
    return _cond(pred, true_fn, false_fn)


def while_loop(cond, body, loop_vars, is_test=False, name=None):  # noqa: A002
    """Reference `layers/control_flow.py` while_loop: concrete values loop eagerly; Program
    Variables record a ``while`` op (condition block + body block, loop-carried variables)."""
    loop_vars = list(loop_vars)
    if any(isinstance(v, Variable) for v in loop_vars):
        from .control_flow import while_loop as _while
        return _while(cond, body, loop_vars)
    while True:
        c = cond(*loop_vars)
        if not (bool(c.reshape(-1)[0]) if isinstance(c, torch.Tensor) else bool(c)):
            break
        out = body(*loop_vars)
        loop_vars = list(out) if isinstance(out, (list, tuple)) else [out]
    return loop_vars


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    xs = x if isinstance(x, (list, tuple)) else [x]
    return _record(func, tuple(xs), {})


from .nn_extra import (case, switch_case, bilinear_tensor_product, conv3d, conv3d_transpose,  # noqa: E402,F401
                       crf_decoding, data_norm, deform_conv2d, nce, row_conv, spectral_norm,
                       multi_box_head, sequence_pool, sequence_first_step, sequence_last_step,
                       sequence_softmax, sequence_concat, sequence_slice, sequence_expand,
                       sequence_expand_as, sequence_pad, sequence_unpad, sequence_reshape,
                       sequence_scatter, sequence_enumerate, sequence_reverse, sequence_conv,
                       StaticRNN)
