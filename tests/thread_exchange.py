"""Test-only Exchange for W emulated ranks as threads of one process (all on one GPU): the same
collective interface as delta_amd.sharded.Exchange, implemented with a barrier and shared slots."""
import threading


class ThreadGroup:
    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world


class ThreadExchange:
    def __init__(self, group, rank):
        self.g, self.rank, self.world = group, rank, group.world

    def _post_and_collect(self, item):
        self.g.slots[self.rank] = item
        self.g.barrier.wait()
        items = list(self.g.slots)
        self.g.barrier.wait()
        return items

    def all_to_all(self, out, inp, out_splits, in_splits):
        import torch
        torch.cuda.current_stream().synchronize()
        items = self._post_and_collect((inp, list(in_splits)))
        pieces = []
        for t, sp in items:
            o = sum(sp[:self.rank])
            pieces.append(t[o:o + sp[self.rank]])
        assert [p.numel() for p in pieces] == list(out_splits)
        if pieces:
            torch.cat(pieces, out=out) if out.numel() else None
        torch.cuda.current_stream().synchronize()
        self._post_and_collect(None)  # sources may be freed only after every rank has copied

    def all_to_all_counts(self, counts, device):
        items = self._post_and_collect(list(counts))
        return [c[self.rank] for c in items]

    def all_reduce_sum(self, vals, device):
        items = self._post_and_collect(list(vals))
        return [sum(v[k] for v in items) for k in range(len(vals))]

    def all_gather_text(self, s):
        return self._post_and_collect(s)

    def barrier(self):
        self.g.barrier.wait()


def run_threads(world, fn):
    """fn(rank, exchange) in `world` threads; returns the per-rank results (re-raises errors)."""
    g = ThreadGroup(world)
    res, err = [None] * world, [None] * world

    def body(r):
        try:
            res[r] = fn(r, ThreadExchange(g, r))
        except BaseException as e:  # noqa: BLE001
            err[r] = e
            g.barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in err:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in err:
        if e is not None:
            raise e
    return res
