import os, sys, tempfile
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ["DR_BA_DEBUG"] = "1"
from delta_amd.testing import synth as S
from delta_amd.delta_log import Engine
d = tempfile.mkdtemp()
exp = S.build_config(3, d, scale=0.005)
eng = Engine.get(0)
staged = eng.stage_log(os.path.join(d, "_delta_log"))
st = staged.replay(exp.min_file_retention_timestamp)
print(st.counts["num_files"], exp.num_files, flush=True)
st.release(); staged.release()
