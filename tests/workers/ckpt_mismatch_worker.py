"""One rank of a sharded checkpoint write whose parts' add rows disagree with numOfFiles (launched by
torch.distributed.run over gloo from tests/test_sharded_cpu.py): every rank must raise the
reference's "State of the checkpoint doesn't match that of the snapshot." (D/Checkpoints.scala:325-328)
instead of leaving the others in the barrier. argv: <log_dir> <out_dir>; rank r writes out_dir/r.txt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


class _Local:
    def write_checkpoint_part(self, part, parts, stats=None, parsed=None, row_group_rows=None, with_adds=False):
        return b"PAR1", 10, 4  # 4 add rows per part: 8 in all against numOfFiles 9


class _Sharded:
    def __init__(self, ex):
        self.exchange = ex
        self.local = _Local()
        from delta_amd.testing import synth as S
        self.nonfile = [{"metaData": S.metadata_dict(2)}]
        self.counts = {"num_files": 9}


def main():
    log_dir, out_dir = sys.argv[1], sys.argv[2]
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from delta_amd.delta_log import DeltaError
    from delta_amd.sharded import Exchange, write_checkpoint_sharded
    ex = Exchange()
    try:
        write_checkpoint_sharded(_Sharded(ex), log_dir, 3)
        outcome = "returned"
    except DeltaError as e:
        outcome = "raised: %s" % e
    with open(os.path.join(out_dir, "%d.txt" % ex.rank), "w") as f:
        f.write(outcome)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
