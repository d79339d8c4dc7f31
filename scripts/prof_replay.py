"""Profiling driver: stages a synthetic config once and runs a few replays (for rocprofv3)."""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    d = os.path.join(tempfile.gettempdir(), "dr_prof_c%d_%g" % (args.config, args.scale))
    if not os.path.exists(os.path.join(d, "_delta_log")):
        S.build_config(args.config, d, scale=args.scale, keep_ids=False, workers=16)
    exp = S.build_config.__module__ and None
    eng = Engine.get(0)
    # context options for the profiled replays: PROF_OPTS="bucket_bits=12,split=0" (dr_ctx_set_option)
    for kv in filter(None, os.environ.get("PROF_OPTS", "").split(",")):
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    staged = eng.stage_log(os.path.join(d, "_delta_log"))
    if os.environ.get("PROF_PLAN"):  # the staged plan's figures (roofline accounting of a profile)
        import json
        print(json.dumps(staged.plan()), flush=True)
    for _ in range(args.reps):
        st = staged.replay(0)
        print(st.counts["num_files"], st.counts["num_actions"], flush=True)
        st.release()
    staged.release()


if __name__ == "__main__":
    main()
