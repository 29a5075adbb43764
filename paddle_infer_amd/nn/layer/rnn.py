"""Recurrent layers: RNN cells, the RNN / BiRNN drivers, multi-layer SimpleRNN / LSTM / GRU, and
beam-search decoding (BeamSearchDecoder + dynamic_decode).

Parity: reference `python/paddle/nn/layer/rnn.py` (RNNCellBase.get_initial_states :151,
SimpleRNNCell, LSTMCell :407 (gates i, f, c, o), GRUCell :564 (reset gate applied after the hidden
matmul), RNN :715, BiRNN :790, SimpleRNN / LSTM / GRU with ``direction`` forward | bidirect,
``time_major``, ``sequence_length`` masking) and `python/paddle/fluid/layers/rnn.py`
(BeamSearchDecoder :871, dynamic_decode :1598, gather_tree).

MI355X-first: the input projection of EVERY time step is one GEMM over the whole sequence
(``[T*B, in] x [in, G*h]`` on hipBLASLt) before the recurrence; the sequential loop only runs the
``[B, h] x [h, G*h]`` hidden projection and the gate elementwise math per step — no per-step
input GEMM, no cuDNN-style packed weight blob.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as TF

from .base import Layer, LayerList
from .. import initializer as I


def _map(fn, x):
    if isinstance(x, (list, tuple)):
        return type(x)(_map(fn, v) for v in x)
    return fn(x)


def _flatten(x):
    if isinstance(x, (list, tuple)):
        out = []
        for v in x:
            out.extend(_flatten(v))
        return out
    return [x]


class RNNCellBase(Layer):
    """Reference `rnn.py:RNNCellBase`: ``get_initial_states`` builds zero (or ``init_value``)
    states shaped by ``state_shape`` with the batch size of ``batch_ref``."""

    def get_initial_states(self, batch_ref, shape=None, dtype=None, init_value=0.0, batch_dim_idx=0):
        ref = _flatten(batch_ref)[0]
        B = ref.shape[batch_dim_idx]
        shape = self.state_shape if shape is None else shape
        dt = dtype if isinstance(dtype, torch.dtype) else ref.dtype

        def make(s):
            s = list(s)
            if s and s[0] == -1:
                s = s[1:]
            return torch.full([B] + s, float(init_value), dtype=dt, device=ref.device)

        def walk(s):
            if isinstance(s, (list, tuple)) and s and isinstance(s[0], (list, tuple)):
                return type(s)(walk(v) for v in s)
            return make(s)
        return walk(shape)

    @property
    def state_shape(self):
        raise NotImplementedError

    @property
    def state_dtype(self):
        return self._dtype

    # cells with a linear input projection run it once over the whole sequence (see RNN)
    # projections on the framework GEMM dispatcher (own 16-bit kernels, split-bf16 fp32 on GPU,
    # forward and backward; torch on CPU)
    def _input_proj(self, x):
        from ...ops.gemm import matmul
        y = matmul(x, self.weight_ih, False, True)
        return y + self.bias_ih if self.bias_ih is not None else y

    def _hidden_proj(self, h):
        from ...ops.gemm import matmul
        y = matmul(h, self.weight_hh, False, True)
        return y + self.bias_hh if self.bias_hh is not None else y

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs, self.state_shape)
        return self._step(self._input_proj(inputs), states)


def _uniform(hidden_size):
    k = 1.0 / math.sqrt(hidden_size)
    return I.Uniform(-k, k)


class _GatedCell(RNNCellBase):
    _gates = 1

    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        if hidden_size <= 0:
            raise ValueError(f"hidden_size of {type(self).__name__} must be greater than 0, got {hidden_size}")
        G = self._gates
        init = _uniform(hidden_size)
        self.weight_ih = self.create_parameter([G * hidden_size, input_size], weight_ih_attr,
                                               default_initializer=init)
        self.weight_hh = self.create_parameter([G * hidden_size, hidden_size], weight_hh_attr,
                                               default_initializer=init)
        self.bias_ih = self.create_parameter([G * hidden_size], bias_ih_attr, is_bias=True,
                                             default_initializer=init)
        self.bias_hh = self.create_parameter([G * hidden_size], bias_hh_attr, is_bias=True,
                                             default_initializer=init)
        self.input_size, self.hidden_size = input_size, hidden_size

    def extra_repr(self):
        return f"{self.input_size}, {self.hidden_size}"


class SimpleRNNCell(_GatedCell):
    """h' = act(W_ih x + b_ih + W_hh h + b_hh), act tanh | relu."""

    def __init__(self, input_size, hidden_size, activation="tanh", weight_ih_attr=None,
                 weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, name=None):
        if activation not in ("tanh", "relu"):
            raise ValueError(f"activation for SimpleRNNCell should be tanh or relu, got {activation}")
        super().__init__(input_size, hidden_size, weight_ih_attr, weight_hh_attr, bias_ih_attr,
                         bias_hh_attr, name)
        self.activation = activation
        self._act = torch.tanh if activation == "tanh" else TF.relu

    def _step(self, xg, h):
        h = self._act(xg + self._hidden_proj(h))
        return h, h

    @property
    def state_shape(self):
        return (self.hidden_size,)


class LSTMCell(_GatedCell):
    """Gates (i, f, c~, o) = split(W_ih x + b_ih + W_hh h + b_hh); c' = f c + i tanh(c~);
    h' = o tanh(c'). States (h, c)."""
    _gates = 4

    def _step(self, xg, states):
        h, c = states
        g = xg + self._hidden_proj(h)
        i, f, cc, o = g.chunk(4, -1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(cc)
        h = torch.sigmoid(o) * torch.tanh(c)
        return h, (h, c)

    @property
    def state_shape(self):
        return ((self.hidden_size,), (self.hidden_size,))


class GRUCell(_GatedCell):
    """r, z = sigmoid(x_r + h_r), sigmoid(x_z + h_z); c = tanh(x_c + r * h_c);
    h' = (h - c) z + c (reset gate applied after the hidden matmul)."""
    _gates = 3

    def _step(self, xg, h):
        hg = self._hidden_proj(h)
        x_r, x_z, x_c = xg.chunk(3, -1)
        h_r, h_z, h_c = hg.chunk(3, -1)
        r = torch.sigmoid(x_r + h_r)
        z = torch.sigmoid(x_z + h_z)
        c = torch.tanh(x_c + r * h_c)
        h = (h - c) * z + c
        return h, h

    @property
    def state_shape(self):
        return (self.hidden_size,)


def _seq_mask(sequence_length, T, dtype, device):
    """[T, B, 1] 1/0 mask of valid steps (time-major)."""
    lens = sequence_length.to(device).reshape(1, -1)
    t = torch.arange(T, device=device).reshape(-1, 1)
    return (t < lens).to(dtype).unsqueeze(-1)


def _run_cell(cell, inputs, states, sequence_length, is_reverse, time_major, **kwargs):
    x = inputs if time_major else inputs.transpose(0, 1)  # [T, B, in]
    T = x.shape[0]
    if states is None:
        states = cell.get_initial_states(x, cell.state_shape, batch_dim_idx=1)
    mask = _seq_mask(sequence_length, T, x.dtype, x.device) if sequence_length is not None else None
    if is_reverse:
        x = x.flip(0)
        mask = mask.flip(0) if mask is not None else None
    fast = hasattr(cell, "_step") and not kwargs
    xg = cell._input_proj(x) if fast else None  # every step's input GEMM at once
    outs = []
    for t in range(T):
        if fast:
            o, new = cell._step(xg[t], states)
        else:
            o, new = cell(x[t], states, **kwargs)
        if mask is not None:
            m = mask[t]
            new = _map_pair(lambda n, s: n * m + s * (1 - m), new, states)
            o = o * m
        states = new
        outs.append(o)
    out = torch.stack(outs, 0)
    if is_reverse:
        out = out.flip(0)
    return (out if time_major else out.transpose(0, 1)), states


def _map_pair(fn, a, b):
    if isinstance(a, (list, tuple)):
        return type(a)(_map_pair(fn, x, y) for x, y in zip(a, b))
    return fn(a, b)


class RNN(Layer):
    """Reference `rnn.py:715`: runs ``cell`` over the time axis; ``sequence_length`` masks padded
    steps (states frozen, outputs zero)."""

    def __init__(self, cell, is_reverse=False, time_major=False):
        super().__init__()
        self.cell = cell
        self.is_reverse, self.time_major = is_reverse, time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        return _run_cell(self.cell, inputs, initial_states, sequence_length, self.is_reverse,
                         self.time_major, **kwargs)


class BiRNN(Layer):
    """Reference `rnn.py:790`: forward and backward cells; outputs concatenated on the feature
    axis, final states ``(fw_states, bw_states)``."""

    def __init__(self, cell_fw, cell_bw, time_major=False):
        super().__init__()
        self.cell_fw, self.cell_bw = cell_fw, cell_bw
        if cell_fw.input_size != cell_bw.input_size:
            raise ValueError("input size of forward cell and backward cell must match")
        self.time_major = time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        s_fw, s_bw = (None, None) if initial_states is None else initial_states
        o_fw, f_fw = _run_cell(self.cell_fw, inputs, s_fw, sequence_length, False, self.time_major, **kwargs)
        o_bw, f_bw = _run_cell(self.cell_bw, inputs, s_bw, sequence_length, True, self.time_major, **kwargs)
        return torch.cat([o_fw, o_bw], -1), (f_fw, f_bw)


class _RNNStack(Layer):
    """Multi-layer (bi)directional SimpleRNN / LSTM / GRU (reference `rnn.py:RNNBase`): a
    LayerList of RNN / BiRNN over cells, dropout between layers; states stacked as
    [num_layers * num_directions, B, h] (LSTM: a (h, c) pair of such)."""
    _cell = None
    _lstm = False

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False,
                 dropout=0.0, activation="tanh", weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        bidir = {"forward": False, "bidirect": True, "bidirectional": True}.get(direction)
        if bidir is None:
            raise ValueError(f"direction should be forward or bidirect (or bidirectional), got {direction}")
        self.num_directions = 2 if bidir else 1
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.time_major, self.dropout = time_major, dropout
        kw = dict(weight_ih_attr=weight_ih_attr, weight_hh_attr=weight_hh_attr,
                  bias_ih_attr=bias_ih_attr, bias_hh_attr=bias_hh_attr)
        if self._cell is SimpleRNNCell:
            kw["activation"] = activation
        layers = []
        for i in range(num_layers):
            isz = input_size if i == 0 else hidden_size * self.num_directions
            if bidir:
                layers.append(BiRNN(self._cell(isz, hidden_size, **kw), self._cell(isz, hidden_size, **kw),
                                    time_major))
            else:
                layers.append(RNN(self._cell(isz, hidden_size, **kw), False, time_major))
        self.layers = LayerList(layers)

    def _split_states(self, initial_states):
        if initial_states is None:
            return [None] * self.num_layers
        nd = self.num_directions
        if self._lstm:
            h, c = initial_states
            per = [(h[i], c[i]) for i in range(h.shape[0])]
        else:
            per = [initial_states[i] for i in range(initial_states.shape[0])]
        return [per[i * nd] if nd == 1 else (per[i * nd], per[i * nd + 1]) for i in range(self.num_layers)]

    def forward(self, inputs, initial_states=None, sequence_length=None):
        states = self._split_states(initial_states)
        x, finals = inputs, []
        for i, layer in enumerate(self.layers):
            if i > 0 and self.dropout > 0 and self.training:
                x = TF.dropout(x, self.dropout)
            x, f = layer(x, states[i], sequence_length)
            finals.extend(f if self.num_directions == 2 else [f])
        if self._lstm:
            return x, (torch.stack([f[0] for f in finals]), torch.stack([f[1] for f in finals]))
        return x, torch.stack(finals)


class SimpleRNN(_RNNStack):
    _cell = SimpleRNNCell


class LSTM(_RNNStack):
    _cell = LSTMCell
    _lstm = True


class GRU(_RNNStack):
    _cell = GRUCell


# ----------------------------------------------------------------------------- decoding
def gather_tree(ids, parents):
    """Reference `gather_tree` op: back-trace beam-search choices. ids / parents [T, B, beam] →
    full token sequences per final beam."""
    T = ids.shape[0]
    out = torch.empty_like(ids)
    beam = torch.arange(ids.shape[2], device=ids.device).expand(ids.shape[1], -1)
    for t in range(T - 1, -1, -1):
        out[t] = ids[t].gather(1, beam)
        beam = parents[t].gather(1, beam)
    return out


class BeamSearchDecoder:
    """Reference `fluid/layers/rnn.py:871`: beam search over an RNN cell. ``embedding_fn`` maps
    token ids to cell inputs, ``output_fn`` maps cell outputs to vocabulary logits."""

    def __init__(self, cell, start_token, end_token, beam_size, embedding_fn=None, output_fn=None):
        self.cell, self.start_token, self.end_token = cell, start_token, end_token
        self.beam_size, self.embedding_fn, self.output_fn = beam_size, embedding_fn, output_fn
        self.kinf = 1e9

    @staticmethod
    def tile_beam_merge_with_batch(x, beam_size):
        """[B, ...] → [B * beam, ...] (each batch entry repeated beam times)."""
        return _map(lambda t: t.unsqueeze(1).expand(t.shape[0], beam_size, *t.shape[1:])
                    .reshape(t.shape[0] * beam_size, *t.shape[1:]), x)

    def _merge(self, x):
        return x.reshape(-1, *x.shape[2:])

    def _split(self, x):
        return x.reshape(-1, self.beam_size, *x.shape[1:])

    def initialize(self, initial_cell_states):
        st = _flatten(initial_cell_states)[0]
        B = st.shape[0]
        dev = st.device
        self.batch_size = B
        self._dev = dev
        cell_states = _map(lambda t: self._split(self.tile_beam_merge_with_batch(t, self.beam_size)),
                           initial_cell_states)
        ids = torch.full((B, self.beam_size), int(self.start_token), dtype=torch.int64, device=dev)
        log_probs = torch.zeros(B, self.beam_size, dtype=torch.float32, device=dev)
        log_probs[:, 1:] = -self.kinf
        finished = torch.zeros(B, self.beam_size, dtype=torch.bool, device=dev)
        lengths = torch.zeros(B, self.beam_size, dtype=torch.int64, device=dev)
        inputs = self.embedding_fn(ids) if self.embedding_fn is not None else ids
        return inputs, {"cell_states": cell_states, "log_probs": log_probs, "finished": finished,
                        "lengths": lengths}, finished

    def step(self, time, inputs, states, **kwargs):
        merged_in = _map(self._merge, inputs)
        merged_states = _map(self._merge, states["cell_states"])
        out, next_cell = self.cell(merged_in, merged_states, **kwargs)
        logits = self.output_fn(out) if self.output_fn is not None else out
        V = logits.shape[-1]
        step_lp = torch.log_softmax(logits.float(), -1).reshape(self.batch_size, self.beam_size, V)
        fin = states["finished"]
        # finished beams only extend with end_token at zero cost
        noend = torch.full((V,), -self.kinf, device=step_lp.device)
        noend[self.end_token] = 0.0
        step_lp = torch.where(fin.unsqueeze(-1), noend, step_lp)
        total = states["log_probs"].unsqueeze(-1) + step_lp
        top, idx = total.reshape(self.batch_size, -1).topk(self.beam_size, -1)
        parent = idx // V
        token = idx % V
        next_cell = _map(lambda t: self._split(t).gather(
            1, parent.reshape(self.batch_size, self.beam_size, *[1] * (t.dim() - 1))
            .expand(-1, -1, *t.shape[1:])), next_cell)
        prev_fin = fin.gather(1, parent)
        lengths = states["lengths"].gather(1, parent) + (~prev_fin).long()
        finished = prev_fin | (token == self.end_token)
        next_states = {"cell_states": next_cell, "log_probs": top, "finished": finished, "lengths": lengths}
        outputs = {"scores": top, "predicted_ids": token, "parent_ids": parent}
        next_inputs = self.embedding_fn(token) if self.embedding_fn is not None else token
        return outputs, next_states, next_inputs, finished

    def finalize(self, outputs, final_states, sequence_lengths):
        ids = gather_tree(outputs["predicted_ids"], outputs["parent_ids"])
        return ids, final_states

    @property
    def tracks_own_finished(self):
        return True


def dynamic_decode(decoder, inits=None, max_step_num=None, output_time_major=False,
                   impute_finished=False, is_test=False, return_length=False, **kwargs):
    """Reference `fluid/layers/rnn.py:1598`: run ``decoder.step`` until every sequence finished
    or ``max_step_num``; returns (final_outputs, final_states[, sequence_lengths]) with outputs
    batch-major unless ``output_time_major``."""
    inputs, states, finished = decoder.initialize(inits)
    outs, t = [], 0
    lengths = None
    while True:
        step_out, next_states, inputs, next_finished = decoder.step(t, inputs, states, **kwargs)
        if impute_finished and not isinstance(states, dict):  # finished entries keep their state
            next_states = _map_pair(lambda n, s: torch.where(
                finished.reshape(-1, *[1] * (n.dim() - 1)), s, n), next_states, states)
        outs.append(step_out)
        states, finished = next_states, next_finished
        t += 1
        if bool(finished.all()) or (max_step_num is not None and t > max_step_num):
            break
    if isinstance(outs[0], dict):
        stacked = {k: torch.stack([o[k] for o in outs], 0) for k in outs[0]}
    else:
        stacked = torch.stack(outs, 0)
    lengths = states.get("lengths") if isinstance(states, dict) else None
    if hasattr(decoder, "finalize"):
        final, states = decoder.finalize(stacked, states, lengths)
    else:
        final = stacked
    if not output_time_major:
        final = _map(lambda x: x.transpose(0, 1) if torch.is_tensor(x) else x, final)
    if return_length:
        return final, states, lengths
    return final, states
