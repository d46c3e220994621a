import os
import socket

import torch


_PORTS_USED = set()


def free_port() -> int:
    """A rendezvous port for spawned ranks: drawn below the kernel's ephemeral range (32768+), so an
    outgoing connection cannot take it between this check and the rank's bind (which the OS-picked
    port 0 allowed: EADDRINUSE flakes), never handed out twice in one test process."""
    import random
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        if p in _PORTS_USED:
            continue
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
        except OSError:
            continue
        finally:
            s.close()
        _PORTS_USED.add(p)
        return p
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class TensorCifar(torch.utils.data.Dataset):
    """Pre-tensorised CIFAR-shaped dataset (no transform RNG): [N,3,32,32] float + int labels."""

    def __init__(self, n, seed=0, learnable=True):
        g = torch.Generator().manual_seed(seed)
        self.targets = torch.randint(0, 10, (n,), generator=g)
        x = torch.randn(n, 3, 32, 32, generator=g) * 0.5
        if learnable:
            x = x + self.targets.view(n, 1, 1, 1).float() * 0.2
        self.x = x
        self.classes = [str(i) for i in range(10)]

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, i):
        return self.x[i], int(self.targets[i])


def dist_env(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
