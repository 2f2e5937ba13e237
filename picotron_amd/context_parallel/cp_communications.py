"""Ring send/recv for context parallelism (API of ref picotron/context_parallel/cp_communications.py:10-54).

Each step posts an isend to the next cp rank and an irecv from the previous one as one batched
P2P (RCCL over xGMI on MI355X); `wait()` waits on the requests only — the reference's extra
device-wide `torch.cuda.synchronize()` (ref :51) is not needed for stream-ordered RCCL P2P.
"""
import os
from typing import List

import torch
import torch.distributed as dist

from .. import process_group_manager as pgm

VERBOSE = os.environ.get("VERBOSE", "0") == "1"


class ContextCommunicate:
    def __init__(self, msg: str = ""):
        self._pending: List[dist.P2POp] = []
        self._active = None
        m = pgm.process_group_manager
        self.rank = m.cp_rank
        self.world_size = m.cp_world_size
        self.send_rank = m.cp_send_rank
        self.recv_rank = m.cp_recv_rank
        self.group = m.cp_group
        self.msg = msg
        if VERBOSE:
            print(f"RingComm ({msg}) | initialized | RANK:{self.rank} | WORLD_SIZE:{self.world_size} | "
                  f"SEND_RANK:{self.send_rank} | RECV_RANK:{self.recv_rank}", flush=True)

    def send_recv(self, tensor_to_send, recv_tensor=None):
        result = (torch.empty(tensor_to_send.shape, dtype=tensor_to_send.dtype, device=tensor_to_send.device)
                  if recv_tensor is None else recv_tensor)
        send_t = tensor_to_send.contiguous()
        self._pending.append(dist.P2POp(dist.isend, send_t, self.send_rank, group=self.group))
        self._pending.append(dist.P2POp(dist.irecv, result, self.recv_rank, group=self.group))
        return result

    def commit(self):
        if self._active is not None:
            raise RuntimeError("Commit called twice")
        self._active = dist.batch_isend_irecv(self._pending)

    def wait(self):
        if self._active is None:
            raise RuntimeError("Wait called before commit")
        for req in self._active:
            req.wait()
        self._active = None
        self._pending = []
