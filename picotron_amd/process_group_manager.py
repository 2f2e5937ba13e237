"""4-D process-group topology (dp, pp, cp, tp), same API as the reference's
picotron/process_group_manager.py:5-68: a module-global `process_group_manager` set by
`setup_process_group_manager(tp_size, cp_size, pp_size, dp_size)`.

The grid is laid out [dp][pp][cp][tp] (tp fastest), as in ref :13; the DP gradient buckets reduce
over `cp_dp_group` (ref :22), which on MI355X is an RCCL communicator over xGMI.
"""
import os

import torch
import torch.distributed as dist

process_group_manager = None


class ProcessGroupManager:
    def __init__(self, tp_size, cp_size, pp_size, dp_size):
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        self.local_rank = int(os.environ.get("LOCAL_RANK", self.global_rank % self.world_size))
        if self.world_size != tp_size * cp_size * pp_size * dp_size:
            raise ValueError(f"World size ({self.world_size}) != TP ({tp_size}) * CP ({cp_size}) * "
                             f"PP ({pp_size}) * DP ({dp_size})")
        grid = torch.arange(self.world_size).view(dp_size, pp_size, cp_size, tp_size)
        self.grid = grid
        self.dp_rank, self.pp_rank, self.cp_rank, self.tp_rank = (grid == self.global_rank).nonzero().flatten().tolist()

        def groups(lists):
            # every rank must create every subgroup in the same order
            return dist.new_subgroups_by_enumeration(lists)[0]

        D, P, C, T = dp_size, pp_size, cp_size, tp_size
        self.tp_group = groups([grid[d, p, c, :].tolist() for d in range(D) for p in range(P) for c in range(C)])
        self.cp_group = groups([grid[d, p, :, t].tolist() for d in range(D) for p in range(P) for t in range(T)])
        self.pp_group = groups([grid[d, :, c, t].tolist() for d in range(D) for c in range(C) for t in range(T)])
        self.dp_group = groups([grid[:, p, c, t].tolist() for p in range(P) for c in range(C) for t in range(T)])
        self.cp_dp_group = groups([grid[:, p, :, t].flatten().tolist() for p in range(P) for t in range(T)])
        self.pp_dp_group = groups([grid[:, :, c, t].flatten().tolist() for c in range(C) for t in range(T)])
        self.world_group = dist.group.WORLD

        d, p, c, t = self.dp_rank, self.pp_rank, self.cp_rank, self.tp_rank
        self.tp_group_ids = grid[d, p, c, :].tolist()
        self.cp_group_ids = grid[d, p, :, t].tolist()
        self.pp_group_ids = grid[d, :, c, t].tolist()
        self.dp_group_ids = grid[:, p, c, t].tolist()
        self.cp_dp_group_ids = grid[:, p, :, t].flatten().tolist()

        self.tp_world_size = dist.get_world_size(group=self.tp_group)
        self.tp_first_rank, self.tp_last_rank = self.tp_group_ids[0], self.tp_group_ids[-1]

        self.cp_world_size = dist.get_world_size(group=self.cp_group)
        self.cp_first_rank, self.cp_last_rank = self.cp_group_ids[0], self.cp_group_ids[-1]
        self.cp_send_rank = self.cp_group_ids[(self.cp_rank + 1) % self.cp_world_size]
        self.cp_recv_rank = self.cp_group_ids[(self.cp_rank - 1) % self.cp_world_size]

        self.pp_world_size = dist.get_world_size(group=self.pp_group)
        self.pp_first_rank, self.pp_last_rank = self.pp_group_ids[0], self.pp_group_ids[-1]
        self.pp_is_first_stage = self.pp_rank == 0
        self.pp_is_last_stage = self.pp_rank == self.pp_world_size - 1
        self.pp_next_rank = None if self.pp_is_last_stage else int(grid[d, p + 1, c, t].item())
        self.pp_prev_rank = None if self.pp_is_first_stage else int(grid[d, p - 1, c, t].item())

        self.dp_world_size = dist.get_world_size(group=self.dp_group)
        self.dp_first_rank, self.dp_last_rank = self.dp_group_ids[0], self.dp_group_ids[-1]
        self.cp_dp_world_size = dist.get_world_size(group=self.cp_dp_group)

    def __str__(self):
        return (f"TP({self.tp_world_size})-CP({self.cp_world_size})-PP({self.pp_world_size})-"
                f"DP({self.dp_world_size})-Rank({self.global_rank})")


def setup_process_group_manager(tp_size, cp_size, pp_size, dp_size):
    global process_group_manager
    process_group_manager = ProcessGroupManager(tp_size, cp_size, pp_size, dp_size)
    return process_group_manager


def tp_world_size():
    return process_group_manager.tp_world_size if process_group_manager is not None else 1


def cp_rank_and_size():
    if process_group_manager is None:
        return 0, 1
    return process_group_manager.cp_rank, process_group_manager.cp_world_size
