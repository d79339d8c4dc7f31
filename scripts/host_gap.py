"""Host-side cost of a replay step: wall time per step against the device time of the same replays
(rocprof-free), with DR_HOST_DEBUG's per-replay host phases (queue / wait / finish) on stderr."""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--timing-only", nargs="*", default=[""],
                    help="per mode: '' no timing, else events on this kernel in every step (bench's timed steps)")
    args = ap.parse_args()
    import torch
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    d = os.path.join(tempfile.gettempdir(), "dr_prof_c3_%g" % args.scale)
    if not os.path.exists(os.path.join(d, "_delta_log")):
        S.build_config(3, d, scale=args.scale, keep_ids=False)
    eng = Engine.get(0)
    staged = eng.stage_log(os.path.join(d, "_delta_log"))
    for _ in range(3):
        staged.replay(0).release()
    for mode in args.timing_only:
        if mode:
            eng.set_timing(True, only=mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            st = staged.replay(0)
            c = st.counts
            st.release()
            if mode:
                eng.last_timings()
        dt = (time.perf_counter() - t0) / args.reps
        eng.set_timing(False)
        print("timing %-16s wall per step %.3f ms (%d reps), files %d" % (mode or "-", dt * 1e3, args.reps,
                                                                          c["num_files"]), flush=True)

if __name__ == "__main__":
    main()
