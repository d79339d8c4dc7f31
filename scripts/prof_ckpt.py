"""Profiling driver for the device checkpoint writer: one part of a config-4 table replayed on the GPU
(DR_CKPT_DEBUG=1 prints the writer's phase times)."""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.01)
    ap.add_argument("--parts", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    d = os.path.join(tempfile.gettempdir(), "dr_prof_ckpt_%g" % args.scale)
    if not os.path.exists(os.path.join(d, "_delta_log")):
        S.build_config(4, d, scale=args.scale, keep_ids=False)
    eng = Engine.get(0)
    staged = eng.stage_log(os.path.join(d, "_delta_log"))
    st = staged.replay(0)
    for r in range(args.reps):
        t0 = time.perf_counter()
        data, rows = st.write_checkpoint_part(1, args.parts)
        print("rep %d: %d rows, %d bytes, %.4f s" % (r, rows, len(data), time.perf_counter() - t0), flush=True)
    st.release()
    staged.release()


if __name__ == "__main__":
    main()
