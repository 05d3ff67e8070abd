"""Debug driver for tests/test_distributed_gpu.py cases: spawns the ranks on
cuda:0 (gloo), each dumping its Python stack if it hangs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch.multiprocessing as mp  # noqa: E402
import test_distributed_gpu as T  # noqa: E402


def w(rank, world, port, case):
    import faulthandler
    faulthandler.dump_traceback_later(60, exit=True)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mpisppy_amd  # noqa: F401
    from mpisppy_amd import _native
    from mpisppy_amd.comm import Comm
    r = T._run_case(case, _native.load(), "cuda:0", mpicomm=Comm())
    print("rank", rank, "iters", r["iters"], r["stats"], flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    case = sys.argv[1]
    world = T.CASES[case][1]
    mp.spawn(w, args=(world, T._free_port(), case), nprocs=world, join=True)
