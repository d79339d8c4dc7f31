"""One rank of a sharded replay (launched by torch.distributed.run from the tests).

argv: <log_path> <cutoff> <out_json> <backend: fake|gpu>
With "fake" the device side is tests/shard_fake.py (CPU, gloo); with "gpu" it is libdeltareplay.
Rank 0 writes the table-wide counters and the gathered records to <out_json>.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    log_path, cutoff, out_path, backend = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    import torch.distributed as dist
    from delta_amd.sharded import Exchange, replay_sharded
    if backend == "fake":
        dist.init_process_group("gloo")
        from tests.shard_fake import FakeHandle, FakeStaged
        ex = Exchange()
        from oracle import delta_oracle as O
        version = O.get_log_segment(log_path).version
        staged = FakeStaged(log_path, ex.world, ex.rank, version)
        st = replay_sharded(staged, cutoff, ex, begin=FakeHandle)
    else:
        import torch
        local = int(os.environ.get("LOCAL_RANK", "0"))
        be = os.environ.get("DR_TEST_BACKEND", "gloo")
        if be == "nccl":  # RCCL: one GPU per rank
            dev = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(be)
        from delta_amd.delta_log import Engine
        from delta_amd.sharded import stage_shard
        ex = Exchange()
        eng = Engine.get(local % max(torch.cuda.device_count(), 1))
        staged = stage_shard(eng, log_path, ex.world, ex.rank)
        st = replay_sharded(staged, cutoff, ex)
    live = st.export_all(0)
    tomb = st.export_all(1)
    if ex.rank == 0:
        with open(out_path, "w") as f:
            json.dump({"counts": st.counts, "nonfile": st.nonfile, "live": live, "tomb": tomb}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
