"""TEST INFRASTRUCTURE: an in-process communicator for ``sirgcn.dist`` — one Python thread per
rank, all on the same device, exchanging rows through shared references.  Lets the -m gpu tests
run the multi-rank halo exchange on device tensors in ONE process (no extra GPU processes).

The autograd engine runs CUDA backward on one thread per device, so rank threads drive
``DistSIRConvFunction.forward/backward`` directly through :class:`FakeCtx` instead of
``Tensor.backward`` (concurrent backward calls with collectives inside would deadlock there)."""
import threading

import torch


class _Shared:
    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world


class ThreadComm:
    def __init__(self, shared, rank):
        self.s, self.rank = shared, rank

    @staticmethod
    def make(world):
        sh = _Shared(world)
        return [ThreadComm(sh, r) for r in range(world)]

    def _sync(self, t):
        if t.is_cuda:
            torch.cuda.synchronize(t.device)
        self.s.barrier.wait()

    def all_to_all_rows(self, out, inp, out_splits, in_splits, async_op=False):
        self.s.slots[self.rank] = (inp, list(in_splits))
        self._sync(inp)
        off = 0
        for q in range(self.s.world):
            src, splits = self.s.slots[q]
            assert splits[self.rank] == out_splits[q], (self.rank, q, splits, out_splits)
            b = sum(splits[:self.rank])
            n = out_splits[q]
            if n:
                out[off:off + n].copy_(src[b:b + n])
            off += n
        self._sync(out)


class FakeCtx:
    """Minimal autograd ctx for calling a Function's static forward/backward by hand."""

    def __init__(self, needs_input_grad):
        self.needs_input_grad = needs_input_grad
        self.saved_tensors = ()

    def save_for_backward(self, *t):
        self.saved_tensors = t


def run_ranks(world, fn):
    """Run fn(rank) on ``world`` threads; re-raise the first failure."""
    out, errs = [None] * world, []

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:      # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    if errs:
        raise errs[0]
    return out


class _Deferred:
    def __init__(self, fn):
        self._fn, self.done = fn, False

    def wait(self):
        if not self.done:
            self._fn()
            self.done = True


class DeferredComm(ThreadComm):
    """Like ThreadComm, but ``async_op=True`` calls return a work object and the rows land only at
    ``wait()`` — until then the destination holds NaN, so a consumer that reads the halo before
    waiting (the stream-ordering bug an async RCCL all-to-all allows) produces NaN."""

    @staticmethod
    def make(world):
        sh = _Shared(world)
        return [DeferredComm(sh, r) for r in range(world)]

    def all_to_all_rows(self, out, inp, out_splits, in_splits, async_op=False):
        if not async_op:
            return super().all_to_all_rows(out, inp, out_splits, in_splits)
        snap = inp.clone()
        out.fill_(float("nan"))
        self.works = getattr(self, "works", 0) + 1
        return _Deferred(lambda: ThreadComm.all_to_all_rows(self, out, snap, out_splits, in_splits))
