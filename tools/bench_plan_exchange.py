"""TP plan-exchange cost: the driver's per-iteration gloo broadcast_object_list of its plan
(engine/engine.py _send_plan) at admission sizes up to 48k prompt tokens, world 2 and 4 (CPU)."""
import os, time, numpy as np, torch, torch.distributed as dist
import torch.multiprocessing as mp
def run(rank, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    for n_tok, n_req in [(0, 0), (1500, 1), (16384, 16), (49152, 48)]:
        ids = np.arange(n_tok, dtype=np.int32)
        plan = {"new": {"ids": ids, "lens": [n_tok // max(n_req,1)] * n_req, "max_new": [300] * n_req,
                        "temp": [0.5] * n_req, "fsm": ["k" * 40] * n_req}, "early": True}
        for _ in range(5):
            box = [plan if rank == 0 else None]; dist.broadcast_object_list(box, src=0)
        t = time.perf_counter(); R = 200
        for _ in range(R):
            box = [plan if rank == 0 else None]; dist.broadcast_object_list(box, src=0)
        dt = (time.perf_counter() - t) / R
        if rank == 0: print(f"world={world} tokens={n_tok:6d} reqs={n_req:3d}: {dt*1e3:.3f} ms per plan")
    dist.destroy_process_group()
if __name__ == "__main__":
    for w in (2, 4):
        mp.spawn(run, args=(w,), nprocs=w)
