"""One rank of the library's RCCL sharded replay (dr_comm_create + dr_replay_sharded), for
tests/test_gpu_sharded.py: rank 0 writes the communicator id to a file, the others read it."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    lp, cutoff, world, rank, uid_file, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        sys.argv[5], sys.argv[6]
    import torch  # noqa: F401  (one HIP runtime: torch's, loaded first)
    from delta_amd.delta_log import DeltaError, Engine
    from delta_amd.sharded import stage_shard
    if rank == 0:
        uid = Engine.comm_unique_id()
        with open(uid_file + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(uid_file + ".tmp", uid_file)
    else:
        t0 = time.time()
        while not os.path.exists(uid_file):
            if time.time() - t0 > 60:
                raise SystemExit("no communicator id")
            time.sleep(0.05)
        with open(uid_file, "rb") as f:
            uid = f.read()
    eng = Engine.get(0)
    try:
        comm = eng.comm(uid, world, rank)
    except DeltaError as e:
        with open(out, "w") as f:
            json.dump({"error": str(e)}, f)
        return
    staged = stage_shard(eng, lp, world, rank)
    st = comm.replay_sharded(staged, cutoff)
    staged.release()
    res = {"counts": st.counts, "nonfile": st.nonfile, "live": st.export(0), "tomb": st.export(1)}
    st.release()
    comm.release()
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
