"""Batch-dimension data parallelism for the multimodal transformer.

The reference is single-process (no DataParallel / NCCL anywhere); this is new.
One process per GPU, full parameter + AdamW replica per rank, each rank draws its own batches
(seed + rank). The per-modality losses are means over B*T (reference model.py:398), so the mean
of the per-rank gradients at equal local batch equals the gradient of the global batch: the
only exchange step is an all-reduce (average) of the flat fp32 gradient.

Overlap: the engine's backward runs in stages (post block, layers L-1..0, embeddings) and the
gradient range of a stage is final once that stage has been enqueued (mmt_backward_stage_range;
every write into a range happens at or before its own stage). `GradSync` groups consecutive
stages into buckets of about `bucket_bytes` and, as soon as a bucket's last stage is enqueued,
issues an async all-reduce of that contiguous slice. With the RCCL ("nccl") backend the
collective runs on the process group's own stream, ordered after the compute already enqueued,
so it proceeds over xGMI while the next stages compute; `finish()` joins the outstanding works
onto the compute stream before the optimizer step.

xGMI is point-to-point (7 links per GPU); RCCL's ring all-reduce is per-link bound, so a few
large buckets (25-50 MB) beat many small ones: at C1 (84 MB of fp32 gradient) that is about
three buckets per step.
"""
import torch
import torch.distributed as dist


def plan_buckets(stage_ranges, bucket_bytes, elem_bytes=4):
    """Group stages (in execution order) into buckets of contiguous parameter ranges.

    stage_ranges: list of (begin, end) in the order the stages run. Returns a list of
    (last_stage_index, [(begin, end), ...]) where each bucket's slices are merged when adjacent.
    A bucket closes once it holds >= bucket_bytes, and always at the last stage.
    """
    buckets = []
    cur, cur_bytes = [], 0
    for s, (b, e) in enumerate(stage_ranges):
        if e > b:
            if cur and cur[-1][0] == e:          # stages walk the layout backwards: merge
                cur[-1] = (b, cur[-1][1])
            elif cur and cur[-1][1] == b:
                cur[-1] = (cur[-1][0], e)
            else:
                cur.append((b, e))
            cur_bytes += (e - b) * elem_bytes
        if cur and (cur_bytes >= bucket_bytes or s == len(stage_ranges) - 1):
            buckets.append((s, cur))
            cur, cur_bytes = [], 0
    return buckets


class GradSync:
    """Bucketed, backward-overlapped gradient averaging over a process group."""

    def __init__(self, stage_ranges, group=None, bucket_bytes=32 << 20):
        self.group = group
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.buckets = plan_buckets(stage_ranges, bucket_bytes)
        self._close = {s: slices for s, slices in self.buckets}
        self._works = []
        self._pending = []

    def _avg_op(self):
        # RCCL supports a native average; gloo does not (sum, then scale in finish())
        return dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM

    def stage_done(self, stage, grad):
        """Call right after stage `stage` of the backward has been enqueued on the current stream."""
        slices = self._close.get(stage)
        if not slices or self.world == 1:
            return
        for b, e in slices:
            t = grad[b:e]
            self._works.append(dist.all_reduce(t, op=self._avg_op(), group=self.group, async_op=True))
            self._pending.append(t)

    def finish(self):
        for w in self._works:
            w.wait()  # NCCL: the current stream waits on the collective; gloo: blocks until done
        if self._avg_op() == dist.ReduceOp.SUM:
            for t in self._pending:
                t.div_(self.world)
        self._works, self._pending = [], []


def enable_data_parallel(model, group=None, bucket_bytes=32 << 20, broadcast=True):
    """Make `model` (a MultimodalTransformer) average its gradient over `group` during backward.

    Broadcasts rank 0's parameters first (identical replicas), then installs a GradSync that the
    model's staged backward drives. Returns the GradSync.
    """
    if broadcast and dist.get_world_size(group) > 1:
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(model.flat_params.data, src=src, group=group)
        if model.flat_unused is not None:
            dist.broadcast(model.flat_unused.data, src=src, group=group)
    sync = GradSync(model.backward_stage_ranges(), group=group, bucket_bytes=bucket_bytes)
    model._grad_sync = sync
    # per-rank dropout stream: every rank seeds torch identically, so without this
    # all ranks would draw the same masks on the same (row, column) sites of their local batches
    model._dp_rank = dist.get_rank()
    return sync
