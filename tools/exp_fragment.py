"""Experiment only: leave the device's memory manager in a fragmented state (many allocations
of random sizes, every other one freed, the rest re-allocated larger, then all freed at exit),
to test whether cfg4's slow mode after other processes follows from physical
placement. GPU box: python tools/exp_fragment.py [GiB]"""
import random
import sys

import torch

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 200
random.seed(5)
held, total = [], 0
while total < gib * 2**30:
    n = random.choice([1, 2, 3, 5, 8, 13, 21, 34, 55]) << 20
    held.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
    total += n
held = held[::2]
torch.cuda.empty_cache()
more, extra = [], 0
while extra < gib / 4 * 2**30:
    n = random.choice([89, 144, 233]) << 20
    more.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
    extra += n
torch.cuda.synchronize()
print("fragmenter: %d + %d allocations held, %.1f GiB reserved" % (len(held), len(more), torch.cuda.memory_reserved() / 2**30))
