"""``paddle.distributed`` (reference `python/paddle/distributed/__init__.py`)."""
from .collective import (ReduceOp, Group, is_initialized, get_rank, get_world_size, new_group,  # noqa: F401
                         get_group, destroy_process_group, all_reduce, broadcast, reduce,
                         all_gather, all_gather_object, reduce_scatter, scatter, alltoall,
                         alltoall_single, send, recv, isend, irecv, P2POp, batch_isend_irecv,
                         barrier, wait, split)
from .parallel import init_parallel_env, ParallelEnv, DataParallel, spawn  # noqa: F401
from . import fleet  # noqa: F401
from .fleet.topology import ParallelMode  # noqa: F401
from .sharding import group_sharded_parallel, save_group_sharded_model  # noqa: F401


def launch():
    from .launch import main
    main()


def gloo_init_parallel_env(rank_id, rank_num, server_endpoint):
    import os
    os.environ.update({"RANK": str(rank_id), "WORLD_SIZE": str(rank_num)})
    host, port = server_endpoint.split(":")
    os.environ.update({"MASTER_ADDR": host, "MASTER_PORT": port})
    return init_parallel_env(backend="gloo")


def gloo_barrier():
    barrier()


def gloo_release():
    destroy_process_group()
from . import checkpoint  # noqa: F401,E402
from .checkpoint import save_state_dict, load_state_dict  # noqa: F401,E402
from . import communication  # noqa: F401,E402
from . import auto_parallel  # noqa: F401,E402
from . import elastic  # noqa: F401,E402
from .auto_parallel import ProcessMesh, shard_tensor, shard_op, reshard  # noqa: F401,E402
from .communication import stream  # noqa: F401,E402
from .dataset import (InMemoryDataset, QueueDataset, CountFilterEntry, ShowClickEntry,  # noqa: F401,E402
                      ProbabilityEntry)
