"""One rank of the host-staged tile test (tests/test_gpu_tiles.py): a column-
strip tile of libgqmap on cuda:0 whose boundary columns and exact totals
travel through torch.distributed gloo (gqmap_tile_exchange_begin / _end).

    python -m tests._tile_host_worker RANK WORLD PORT ITS OUT.npz
"""
import os
import sys

import numpy as np


def main():
    rank, world, port, its, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import torch
    import torch.distributed as dist
    from gqmap_opticalflow_amd import Engine
    from tests.test_gpu_tiles import _problem
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        I1, I2, o = _problem("mixture", 3, 96, 128)
        e = Engine(o, I1, I2, "mixture", "fp64", device=0, n_tiles=world, tile=rank)
        e.attach_host()
        e.init_state(3)
        traces = []
        for _ in range(its):
            sl, sr, tot = e.exchange_begin()
            bufs, reqs = {}, []
            if rank > 0:  # my first owned column -> left; its last owned column <- left
                bufs["l"] = torch.empty(e.xfer_sizes[2], dtype=torch.uint8)
                reqs += [dist.isend(torch.from_numpy(sl), rank - 1), dist.irecv(bufs["l"], rank - 1)]
            if rank < world - 1:
                bufs["r"] = torch.empty(e.xfer_sizes[3], dtype=torch.uint8)
                reqs += [dist.isend(torch.from_numpy(sr), rank + 1), dist.irecv(bufs["r"], rank + 1)]
            for r in reqs:
                r.wait()
            allt = [torch.empty(tot.size, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(allt, torch.from_numpy(tot))
            tr = e.exchange_end(bufs["l"].numpy() if "l" in bufs else None,
                                bufs["r"].numpy() if "r" in bufs else None,
                                torch.cat(allt).numpy())
            traces.append(tr)
        st = e.get_state()
        np.savez(out, col0=e.col0, col1=e.col1, trace=np.array(traces),
                 **{k: getattr(st, k)[:, e.col0:e.col1] for k in ("muu", "muv", "sigu", "sigv", "pn", "rou")},
                 alpha=st.alpha, w=st.w)
        e.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
