"""HybridParallelInferenceHelper: split a static inference program over pipeline stages (and
model-parallel rings) for multi-rank serving.

Parity: reference `python/paddle/distributed/fleet/utils/hybrid_parallel_inference.py:23`. Ops are
placed with ``paddle.static.device_guard("gpu:<stage>")`` (``"gpu:all"`` / untagged: every stage);
ranks form a [num_pp, num_mp] grid (stage = row, model-parallel slice = column), ring 0 is this
rank's model-parallel group (the ``c_allreduce_sum`` / ``c_identity`` ops of tensor-parallel layers
run on it) and ring 1 the global ring.

``gen_infer_program`` rewrites the program in place for THIS rank, walking every block in program
order identically on all ranks so the inserted collectives pair up:

* an op of another stage is dropped;
* a value produced on stage p and read by an op of stage s ≠ p gets ``send_v2`` on p and
  ``recv_v2`` on s at the reader's position (once per value version and stage);
* a value produced on stage p and read by an every-stage op (e.g. the loop condition) is
  ``c_broadcast`` from p over the pipeline ring;
* at the end of every ``while`` body the loop-carried results (and the names passed in
  ``sync_in_while_lastpp2firstpp_var_names`` / ``sync_in_while_var_names``) are broadcast from the
  stage that computed them, so every stage enters the next iteration — and evaluates the
  condition — on the same values.

Fetch targets live on the stage that computes them (the last stage for a model output).
"""
from __future__ import annotations

import numpy as np

from ...static.framework import Operator

PP_RING = 2  # the pipeline-column ring the helper binds for its broadcasts


def _stage_of(op):
    d = op.attrs.get("op_device")
    if d is None or not isinstance(d, str) or d.endswith(":all") or ":" not in d:
        return None
    return int(d.split(":")[1])


def _new(block, t, ins, outs, attrs):
    op = Operator(block, None, (), {}, None, type=t, attrs=attrs)
    op.paddle_inputs, op.paddle_outputs = ins, outs
    return op


class HybridParallelInferenceHelper:
    def __init__(self, startup_program, main_program, num_mp=1, num_pp=1, micro_batch_size=1,
                 beam_size=1, init_comm=True, role_maker=None):
        import torch.distributed as dist
        self._startup_program, self._main_program = startup_program, main_program
        self.num_mp, self.num_pp = int(num_mp), int(num_pp)
        self.micro_batch_size, self.beam_size, self.init_comm = micro_batch_size, beam_size, init_comm
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.nranks = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if self.num_mp * self.num_pp != self.nranks:
            raise ValueError(f"num_mp ({num_mp}) x num_pp ({num_pp}) != world size {self.nranks}")
        arr = np.arange(self.nranks).reshape(self.num_pp, self.num_mp)
        ipp, imp = [int(v[0]) for v in np.where(arr == self.rank)]
        self.mp_group = [int(r) for r in arr[ipp, :]]
        self.pp_group = [int(r) for r in arr[:, imp]]
        self._stage = ipp
        self._grid = arr
        self.mp_ring_id, self.global_ring_id = 0, 1

    # ------------------------------------------------------------------ communicators
    def _init_communication_group(self):
        from .. import collective as C
        if self.nranks == 1:
            return
        for row in self._grid:  # new_group is collective: every rank creates every group
            g = C.new_group([int(r) for r in row])
            if self.rank in row:
                C.bind_ring(self.mp_ring_id, g)
        C.bind_ring(self.global_ring_id, C.new_group(list(range(self.nranks))))
        for col in self._grid.T:
            g = C.new_group([int(r) for r in col])
            if self.rank in col:
                C.bind_ring(PP_RING, g)

    # ------------------------------------------------------------------ rewriting
    def _bcast(self, block, name, src_stage):
        return _new(block, "c_broadcast", {"X": [name]}, {"Out": [name]},
                    {"ring_id": PP_RING, "root": int(src_stage), "use_calc_stream": True})

    def _split_block(self, block, producer, extra_sync=()):
        """Rewrite ``block`` for this rank; ``producer``: var → stage (None = every stage)."""
        prog = block.program
        me = self._stage
        out = []
        delivered = set()
        for op in list(block.ops):
            st = _stage_of(op)
            needs = []
            for v in op.input_names():
                p = producer.get(v)
                if p is not None and p != st:
                    needs.append((v, p))
            for v, p in sorted(set(needs)):
                if st is None:  # every stage reads it: broadcast from its producer
                    out.append(self._bcast(block, v, p))
                    producer[v] = None
                elif (v, st) not in delivered:
                    if me == p:
                        out.append(_new(block, "send_v2", {"X": [v]}, {},
                                        {"ring_id": self.global_ring_id, "peer": self.pp_group[st],
                                         "use_calc_stream": True}))
                    if me == st:
                        out.append(_new(block, "recv_v2", {}, {"Out": [v]},
                                        {"ring_id": self.global_ring_id, "peer": self.pp_group[p],
                                         "use_calc_stream": True}))
                    delivered.add((v, st))
            if op.func is None and op.type in ("while", "cond"):
                for key in ("cond_block", "body_block", "true_block", "false_block"):
                    if key in op.attrs:
                        sub = prog.block(op.attrs[key])
                        sync = ()
                        if key == "body_block":
                            sync = tuple(op.attrs.get("body_outs", [])) + tuple(extra_sync)
                        self._split_block(sub, producer, sync)
                # the loop's / branch's results exist on every stage (synced in the body)
                for n in op.output_names():
                    producer[n] = None
                out.append(op)
                continue
            if st is None or st == me:
                out.append(op)
            for n in op.output_names():
                producer[n] = st
                delivered = {d for d in delivered if d[0] != n}
        for v in dict.fromkeys(extra_sync):  # end of a loop body: every stage gets the results
            p = producer.get(v)
            if p is not None:
                out.append(self._bcast(block, v, p))
                producer[v] = None
        block.ops[:] = out
        for i, op in enumerate(block.ops):
            op.idx = i
        prog._version += 1

    def gen_infer_program(self, sync_in_while_lastpp2firstpp_var_names=None,
                          sync_in_while_var_names=None, debug=False):
        if self.init_comm:
            self._init_communication_group()
        if self.num_pp == 1:
            return
        extra = list(sync_in_while_lastpp2firstpp_var_names or []) + list(sync_in_while_var_names or [])
        self._split_block(self._main_program.global_block(), {}, ())
        if extra:  # user-listed loop values: broadcast at the end of every while body as well
            for b in self._main_program.blocks[1:]:
                producer = {}
                for op in b.ops:
                    for n in op.output_names():
                        producer[n] = _stage_of(op)
                for v in extra:
                    if v in producer and producer[v] is not None and not any(
                            o.type == "c_broadcast" and o.paddle_outputs.get("Out") == [v] for o in b.ops):
                        b.ops.append(self._bcast(b, v, producer[v]))
        if debug:
            for i, b in enumerate(self._main_program.blocks):
                print(f"[rank {self.rank} stage {self._stage}] block {i}:",
                      [o.type for o in b.ops], flush=True)
