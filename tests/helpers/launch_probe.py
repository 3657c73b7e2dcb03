"""Rank body for tests/test_bench_launch.py: what a bench.py rank does before its GPU
work — read the launcher's RANK / WORLD_SIZE / MASTER_*, join the process group (gloo on
the CPU), all-gather the rank topology (bench.rank_topology) and have rank 0 print one
JSON line. Run only through bench.self_launch."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    import bench
    world = int(os.environ["WORLD_SIZE"])
    bench.join_group(dist, "gloo", None, float(os.environ.get("PROBE_RDZV_TIMEOUT", "120")))
    ranks, backend = bench.rank_topology(dist, torch.device("cpu"), world)
    t = torch.tensor([float(dist.get_rank() + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # what this rank of `bench.py --gpus world` fits (no --segments; config 4 splits 10M evenly)
    plan = bench.plan_workload(world) if bench.CONFIG4_SEGMENTS % world == 0 else {"workload": None,
                                                                                   "record_segments": None}
    if dist.get_rank() == 0:
        print(json.dumps({"n_gpus": world, "world": {"size": world, "backend": backend, "ranks": ranks},
                          "max_over_ranks": float(t.item()), "argv": sys.argv[1:],
                          "config": {"workload": plan["workload"], "record_segments": plan["record_segments"]}}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
