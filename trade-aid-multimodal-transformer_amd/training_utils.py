"""training_utils.py — drop-in for the reference's batch generation, evaluation loop and
directional metric (reference training_utils.py:33-534), re-designed for a GPU step rate.

Same public names, arguments, module globals (set by main.py, reference main.py:387-396), print
lines and log lines. What changed underneath:
  * generate_batch_starting_indices draws its indices with the SAME torch.randint calls as the
    reference (bit-identical under a seeded torch RNG) but maps them to file positions with a
    vectorised searchsorted instead of a per-sample Python loop (training_utils.py:156-178);
  * get_batch keeps the reference's in-place +-1 random walk of the training set, driven by
    all_modality_params[r][2] (`has_header`, the reference quirk at training_utils.py:353; see
    DESIGN.md). Two modes:
      - exact (use_device_batcher = False, or MMT_EXACT_BATCHER=1): numpy over the host int64
        streams, bit-exact with the reference including its consumption of Python's `random`
        (jitter_exact_) and torch's CPU generator (start indices); the windows go to the GPU
        through pinned host buffers (non_blocking copies);
      - fast (default on a GPU): DeviceBatcher, the streams resident in HBM and the walk, the
        start indices and the gather as HIP kernels driven by a counter hash: the same laws
        (tested), not the same draws;
      - exact on the device (batcher_mode = "exact", or MMT_EXACT_BATCHER=device):
        ExactDeviceBatcher, bit-exact like the host mode at device speed: the streams resident in
        HBM, Python's MT19937 run on the GPU from random.getstate() (mmt_exact_gen, a side stream,
        overlapping the previous step) and the walk as prefix-sum kernels (mmt_exact_walk); the
        start indices drawn with the reference's torch.randint calls on the CPU (a few dozen
        values), the windows gathered on the device. Python's `random` state and the host
        training lists are brought up to date at every estimate_loss and by sync_host_state();
  * calculate_evaluation_metrics runs the per-sample argmax / direction / softmax-certainty loop
    (training_utils.py:259-304) as one HIP kernel per modality (mmt_eval_direction) with a single
    device->host copy, instead of B*V `.item()` syncs.
"""
import ctypes
import math
import numbers
import os
import random
from datetime import datetime

import numpy as np
import torch

import mmt_lib as ML
from config_utils import _get_batch_size, _get_block_size, _get_config, _get_device, _get_eval_iters

__all__ = ["generate_batch_starting_indices", "get_batch", "estimate_loss", "calculate_evaluation_metrics"]


# ------------------------------------------------------------------------------------------
# batch start indices (reference training_utils.py:33-181)
# ------------------------------------------------------------------------------------------
def _split_file_lengths(data_size, split, file_lengths):
    lens = []
    acc = 0
    n = len(file_lengths)
    for f in range(n):
        this = file_lengths[f] if split == "train" else file_lengths[n - 1 - f]
        acc += this
        if acc <= data_size:
            lens.append(this)
        if acc > data_size:
            lens.append(data_size - (acc - this))
        if acc >= data_size:
            if split == "val":
                lens.reverse()
            break
    return lens


def generate_batch_starting_indices(data_size, block_size, batch_size, split, file_lengths, is_percents):
    """Random start indices whose [i, i+block_size] window stays inside one file of the split."""
    if not isinstance(data_size, int) or data_size <= 0:
        raise TypeError("'data_size' must be a positive integer.")
    if not isinstance(block_size, int) or block_size <= 0:
        raise TypeError("'block_size' must be a positive integer.")
    if block_size >= data_size:
        raise ValueError("'block_size' cannot be equal to or greater than 'data_size'.")
    if not isinstance(batch_size, int) or batch_size <= 0:
        raise TypeError("'batch_size' must be a positive integer.")
    if not isinstance(split, str) or split not in ("train", "val"):
        raise ValueError("'split' must be 'train' or 'val'.")
    if not isinstance(file_lengths, list) or not len(file_lengths) >= 1:
        raise TypeError("'file_lengths' must be a list containing at least 1 element.")
    if not isinstance(is_percents, bool):
        raise TypeError("'is_percents' must be a boolean.")
    bxy = block_size + 1
    off = 1 if is_percents else 0
    if len(file_lengths) == 1:
        return torch.randint(off, data_size - bxy + 1, (batch_size,))
    lens = np.asarray(_split_file_lengths(data_size, split, file_lengths), dtype=np.int64)
    valid = np.maximum(0, lens - bxy - off + 1)
    total = int(valid.sum())
    if total <= 0:
        raise ValueError("No valid starting positions available for the given block size and file lengths.")
    init = torch.randint(total, (batch_size,)).numpy()
    cum_valid = np.cumsum(valid)
    k = np.searchsorted(cum_valid, init, side="right")  # first file whose cumulative count exceeds init
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    prev = np.concatenate([[0], cum_valid[:-1]])
    return torch.from_numpy(starts[k] + (init - prev[k]) + off).to(torch.long)


# ------------------------------------------------------------------------------------------
# get_batch (reference training_utils.py:333-384 + data_utils.py:293-358)
# ------------------------------------------------------------------------------------------
_pinned = {}


def _as_array(r):
    """Train sets arrive as Python lists (reference main.py:374). Convert once, IN PLACE in the
    shared list object, so the random walk keeps mutating the one training set as in the reference."""
    t = all_train_sets[r]
    if isinstance(t, np.ndarray):
        return t
    arr = np.asarray(t.tolist() if isinstance(t, torch.Tensor) else t, dtype=np.int64)
    all_train_sets[r] = arr
    return arr


_CHOICES = np.array([0, 1, -1, 2, -2, 3, -3], dtype=np.int64)  # rand_list of data_utils.py:342-345


def _mt_from_python(state):
    """numpy MT19937 positioned exactly where Python's `random` is (same key words and index:
    CPython's Random is MT19937 and getrandbits(k <= 32) is one genrand_uint32() >> (32 - k))."""
    bg = np.random.MT19937()
    bg.state = {"bit_generator": "MT19937",
                "state": {"key": np.asarray(state[1][:624], dtype=np.uint32), "pos": int(state[1][624])}}
    return bg


def jitter_exact_(arrs, rand_sizes, vocab_sizes, pyrandom=random):
    """add_rand_to_data_points (reference data_utils.py:342-351) over several training streams in
    the order get_batch calls it (training_utils.py:352-360), bit-exact with the reference's
    Python loop AND its consumption of Python's global `random` stream, vectorised.

    Reference: every element x with r < x < V - r (r = rand_size, read from the eligibility BEFORE
    this pass: an element is visited once) gets x += random.choice(rand_list), rand_list =
    [0, 1, -1, .., r, -r]. random.choice(seq) is seq[_randbelow(len(seq))] and _randbelow(n) draws
    getrandbits(n.bit_length()) until the value is < n (CPython 3.x). So the eligible elements,
    stream by stream, take the accepted values of one MT19937 sequence in order. This draws that
    sequence with numpy's MT19937 from `random.getstate()`, stops exactly at the last draw the loop
    would make, and writes the advanced state back into `random`."""
    jobs = []
    for arr, rs, V in zip(arrs, rand_sizes, vocab_sizes):
        if rs is None:
            continue
        if not isinstance(rs, (int, np.integer)):
            raise TypeError("rand_size must be an integer or null.")
        r = int(rs)
        if r < 1 or r > 3:
            raise ValueError("rand_size must be an integer between 1 and 3, or null.")
        if not isinstance(V, (int, np.integer)) or V <= 0:
            raise TypeError("vocab_size must be a positive integer.")
        elig = np.flatnonzero((arr > r) & (arr < int(V) - r))
        jobs.append((arr, elig, 2 * r + 1))
    need = sum(len(e) for _, e, _ in jobs)
    if need == 0:
        return
    state = pyrandom.getstate()
    bg = _mt_from_python(state)
    # every job's n = 2r+1 has the same bit length only when the rand sizes agree; walk per job
    for arr, elig, n in jobs:
        m = len(elig)
        if m == 0:
            continue
        k = int(n).bit_length()
        got = []
        have = 0
        chunk = m  # each accepted value needs >= 1 draw
        while have < m:
            saved = bg.state
            raw = bg.random_raw(chunk) >> np.uint64(32 - k)
            acc = np.flatnonzero(raw < np.uint64(n))
            if have + len(acc) >= m:
                take = m - have
                used = int(acc[take - 1]) + 1  # the loop stops right after the m-th accepted draw
                bg.state = saved
                bg.random_raw(used)
                got.append(raw[acc[:take]])
                have = m
            else:
                got.append(raw[acc])
                have += len(acc)
                chunk = max(1024, (m - have) * 3 // 2)
        vals = np.concatenate(got).astype(np.int64)
        arr[elig] += _CHOICES[vals]
    st = bg.state["state"]
    pyrandom.setstate((state[0], tuple(int(x) for x in st["key"]) + (int(st["pos"]),), state[2]))


_RING = 4
_ring_pos = [0]
_ring_events = [None] * _RING


def _pinned_buf(key, shape):
    b = _pinned.get(key)
    if b is None or tuple(b.shape) != tuple(shape):
        b = torch.empty(shape, dtype=torch.long, pin_memory=torch.cuda.is_available())
        _pinned[key] = b
    return b


def _ring_slot():
    """Pick the next pinned-buffer set; wait only for the async H2D copy issued from it _RING calls ago."""
    slot = _ring_pos[0]
    _ring_pos[0] = (slot + 1) % _RING
    ev = _ring_events[slot]
    if ev is not None:
        ev.synchronize()
    return slot


class DeviceBatcher:
    """get_batch for token streams resident in HBM: the training streams live on the GPU as int32,
    the +-r random walk, the start indices and the window gather are HIP kernels
    (mmt_batch_jitter / mmt_batch_indices / mmt_batch_gather): no host work, no PCIe per step."""

    def __init__(self, train_sets, val_sets, vocab_sizes, rand_sizes, file_lengths, is_percents, block_size,
                 batch_size, device, seed=0):
        self.device = torch.device(device)
        self.T, self.B = int(block_size), int(batch_size)
        self.rand = list(rand_sizes)
        self.V = [int(v) for v in vocab_sizes]
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.counter = 0

        def dev32(a):
            a = a.numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
            return torch.from_numpy(a.astype(np.int32)).to(self.device)

        self.data = {"train": [dev32(t) for t in train_sets], "val": [dev32(v) for v in val_sets]}
        self.maps = {}
        bxy = self.T + 1
        off = 1 if is_percents else 0
        for split in ("train", "val"):
            n = int(self.data[split][0].numel())
            if len(file_lengths) == 1:
                lens = np.array([n], dtype=np.int64)
                valid = np.array([max(0, n - bxy - off + 1)], dtype=np.int64)
            else:
                lens = np.asarray(_split_file_lengths(n, split, file_lengths), dtype=np.int64)
                valid = np.maximum(0, lens - bxy - off + 1)
            if valid.sum() <= 0:
                raise ValueError("No valid starting positions available for the given block size and file lengths.")
            starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            self.maps[split] = (torch.from_numpy(np.cumsum(valid)).to(self.device),
                                torch.from_numpy(starts).to(self.device), len(lens), off)

    def next(self, split, is_training):
        L = ML.lib()
        s = ML.stream_ptr(self.device)
        self.counter += 1
        if is_training == 1:
            for r, t in enumerate(self.data["train"]):
                if self.rand[r] is not None:
                    ML.check(L.mmt_batch_jitter(s, ML.ptr(t), t.numel(), int(self.rand[r]), self.V[r], self.seed,
                                                self.counter * 64 + r), None, "mmt_batch_jitter")
        cum, starts, nf, off = self.maps[split]
        ix = torch.empty(self.B, dtype=torch.long, device=self.device)
        ML.check(L.mmt_batch_indices(s, self.B, ML.ptr(cum), ML.ptr(starts), nf, off, self.seed ^ 0x5EED,
                                     self.counter, ML.ptr(ix)), None, "mmt_batch_indices")
        data = self.data[split]
        xs = [torch.empty(self.B, self.T, dtype=torch.long, device=self.device) for _ in data]
        ys = [torch.empty(self.B, self.T, dtype=torch.long, device=self.device) for _ in data]
        ML.check(L.mmt_batch_gather(s, len(data), ML.ptr_array(data), ML.ptr(ix), self.B, self.T, ML.ptr_array(xs),
                                    ML.ptr_array(ys)), None, "mmt_batch_gather")
        return xs, ys


class ExactDeviceBatcher:
    """get_batch bit-exact with the reference (walk, Python `random` consumption, torch start
    indices) with the token streams resident in HBM: see the module docstring and
    csrc/mmt_batch.hip (mmt_exact_gen / mmt_exact_walk)."""

    def __init__(self, train_sets, val_sets, vocab_sizes, rand_sizes, file_lengths_, is_percents_, block_size,
                 batch_size, device):
        self.device = torch.device(device)
        self.T, self.B = int(block_size), int(batch_size)
        self.file_lengths, self.is_percents = file_lengths_, bool(is_percents_)
        self.V = [int(v) for v in vocab_sizes]
        rs = []
        for r in rand_sizes:  # the reference's checks (data_utils.py:322-330)
            if r is None:
                rs.append(0)
                continue
            if not isinstance(r, (int, np.integer)):
                raise TypeError("rand_size must be an integer or null.")
            if int(r) < 1 or int(r) > 3:
                raise ValueError("rand_size must be an integer between 1 and 3, or null.")
            rs.append(int(r))
        self.rs = rs
        self.host_train = train_sets

        def dev32(a):
            a = a.numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
            return torch.from_numpy(a.astype(np.int32)).to(self.device)

        self.data = {"train": [dev32(_as_array(i)) for i in range(len(train_sets))],
                     "val": [dev32(v) for v in val_sets]}
        n = [int(t.numel()) for t in self.data["train"]]
        # words per step: every element eligible, 2% over the expected draws + a fixed margin (the
        # shortfall probability is astronomically small; the walk flags it in self.status)
        self.nwords = 16384 + sum(int(math.ceil(ni * (1 << (2 * r + 1).bit_length()) / (2 * r + 1) * 1.02))
                                  for ni, r in zip(n, rs) if r)
        L = ML.lib()
        self.words = torch.empty(max(1, L.mmt_exact_words_bytes(self.nwords)) // 4, dtype=torch.int32,
                                 device=self.device)
        self.scratch = torch.empty(L.mmt_exact_walk_scratch_bytes(max(n + [1]), self.nwords), dtype=torch.uint8,
                                   device=self.device)
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.n = (ctypes.c_int64 * len(n))(*n)
        self.rs_c = (ctypes.c_int32 * len(rs))(*rs)
        self.V_c = (ctypes.c_int32 * len(self.V))(*self.V)
        self._load_state(random.getstate())
        self.side = torch.cuda.Stream(device=self.device)
        self.gen_done = None  # event: the words of the next walk are generated
        self.dirty = False    # device walk / generator state ahead of the host copies

    def _load_state(self, st):
        key = np.asarray(st[1], dtype=np.uint32)  # 624 key words + index
        self.mt = torch.from_numpy(key.view(np.int32).copy()).to(self.device)
        self.py_state = st

    def _gen(self, stream):
        ML.check(ML.lib().mmt_exact_gen(ML.stream_ptr(self.device, stream), ML.ptr(self.mt), ML.ptr(self.words),
                                        self.nwords), None, "mmt_exact_gen")

    def next(self, split, is_training):
        L = ML.lib()
        cur = torch.cuda.current_stream(self.device)
        if is_training == 1 and any(self.rs):
            if random.getstate() != self.py_state:
                raise RuntimeError("Python's `random` was used between device-exact get_batch calls: the reference "
                                   "shares that stream with its walk; call training_utils.sync_host_state() first")
            if self.gen_done is None:
                self._gen(cur)
            else:
                cur.wait_event(self.gen_done)
            ptrs = (ctypes.c_void_p * len(self.rs))(*[t.data_ptr() for t in self.data["train"]])
            ML.check(L.mmt_exact_walk(ML.stream_ptr(self.device, cur), len(self.rs), ptrs, self.n, self.rs_c, self.V_c,
                                      ML.ptr(self.mt), ML.ptr(self.words), self.nwords, ML.ptr(self.scratch),
                                      self.scratch.numel(), ML.ptr(self.status)), None, "mmt_exact_walk")
            # the next step's words, generated on the side stream while this step computes
            ev = torch.cuda.Event()
            ev.record(cur)
            self.side.wait_event(ev)
            self._gen(self.side)
            self.gen_done = torch.cuda.Event()
            self.gen_done.record(self.side)
            self.dirty = True
        data = self.data[split]
        ix = generate_batch_starting_indices(int(data[0].numel()), self.T, self.B, split, self.file_lengths,
                                             self.is_percents)  # the reference's torch.randint calls
        slot = _ring_slot()
        ixp = _pinned_buf(("ix", slot), (self.B,))
        ixp.copy_(ix)
        ixd = ixp.to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cur)
        _ring_events[slot] = ev
        xs = [torch.empty(self.B, self.T, dtype=torch.long, device=self.device) for _ in data]
        ys = [torch.empty(self.B, self.T, dtype=torch.long, device=self.device) for _ in data]
        ML.check(L.mmt_batch_gather(ML.stream_ptr(self.device, cur), len(data), ML.ptr_array(data), ML.ptr(ixd), self.B,
                                    self.T, ML.ptr_array(xs), ML.ptr_array(ys)), None, "mmt_batch_gather")
        return xs, ys

    def sync_host_state(self):
        """Python's `random` state and the walked training lists (in place) as the reference's loop
        leaves them; one device sync."""
        if not self.dirty:
            return
        if int(self.status.item()):
            raise RuntimeError("device-exact get_batch: the generated MT19937 words ran out (walk incomplete)")
        key = self.mt.cpu().numpy().view(np.uint32)
        st = (self.py_state[0], tuple(int(x) for x in key), self.py_state[2])
        random.setstate(st)
        self.py_state = random.getstate()
        for i, t in enumerate(self.data["train"]):
            arr = _as_array(i)
            arr[...] = t.cpu().numpy()
        self.dirty = False


_device_batcher = [None]
use_device_batcher = os.environ.get("MMT_EXACT_BATCHER", "0") in ("", "0", "device")
# "hash": DeviceBatcher (counter-hash draws, same laws), "exact": ExactDeviceBatcher (bit-exact)
batcher_mode = "exact" if os.environ.get("MMT_EXACT_BATCHER", "") == "device" else "hash"


def _get_device_batcher():
    b = _device_batcher[0]
    key = (id(all_train_sets), id(all_val_sets), _get_block_size(), _get_batch_size(), str(_get_device()), batcher_mode)
    if b is None or b[0] != key:
        if b is not None and isinstance(b[1], ExactDeviceBatcher):
            b[1].sync_host_state()
        if batcher_mode == "exact":
            inst = ExactDeviceBatcher(all_train_sets, all_val_sets, [len(v) for v in all_vocabularies],
                                      [p[2] for p in all_modality_params], file_lengths, is_percents,
                                      _get_block_size(), _get_batch_size(), _get_device())
        else:
            inst = DeviceBatcher(all_train_sets, all_val_sets, [len(v) for v in all_vocabularies],
                                 [p[2] for p in all_modality_params], file_lengths, is_percents, _get_block_size(),
                                 _get_batch_size(), _get_device(), seed=random.getrandbits(63))
        b = (key, inst)
        _device_batcher[0] = b
    return b[1]


def sync_host_state():
    """Device-exact mode: write the device's walk and generator state back into the training lists
    and Python's `random` (as the reference's loop leaves them); a no-op in the other modes."""
    b = _device_batcher[0]
    if b is not None and isinstance(b[1], ExactDeviceBatcher):
        b[1].sync_host_state()


def get_batch(split, is_training):
    """Returns (xb_list, yb_list), each M tensors [batch_size, block_size] int64 on the device."""
    T = _get_block_size()
    B = _get_batch_size()
    dev = _get_device()
    if use_device_batcher and dev != "cpu" and torch.cuda.is_available():
        return _get_device_batcher().next(split, is_training)
    if is_training == 1:
        # reference quirk: the jitter size is all_modality_params[r][2] (has_header), not index 7
        jitter_exact_([_as_array(r) for r in range(num_modalities)],
                      [all_modality_params[r][2] for r in range(num_modalities)],
                      [len(all_vocabularies[r]) for r in range(num_modalities)])
    if split == "train":
        data = [_as_array(r) for r in range(num_modalities)]
    else:
        data = [v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v) for v in all_val_sets]
    ix = generate_batch_starting_indices(len(data[0]), T, B, split, file_lengths, is_percents).numpy()
    win = ix[:, None] + np.arange(T + 1)[None, :]
    xb_list, yb_list = [], []
    on_gpu = dev != "cpu" and torch.cuda.is_available()
    slot = _ring_slot() if on_gpu else 0
    for r in range(num_modalities):
        w = data[r][win]
        xb = _pinned_buf(("x", r, slot), (B, T))
        yb = _pinned_buf(("y", r, slot), (B, T))
        xb.numpy()[...] = w[:, :T]
        yb.numpy()[...] = w[:, 1:]
        if on_gpu:
            xb_list.append(xb.to(dev, non_blocking=True))
            yb_list.append(yb.to(dev, non_blocking=True))
        else:
            xb_list.append(xb.clone())
            yb_list.append(yb.clone())
    if on_gpu:
        ev = torch.cuda.Event()
        ev.record()
        _ring_events[slot] = ev
    return xb_list, yb_list


# ------------------------------------------------------------------------------------------
# directional metric (reference training_utils.py:184-330)
# ------------------------------------------------------------------------------------------
_vocab_dev = {}


def _get_direction_sign(current_value, previous_value, is_percentage_data):
    if is_percentage_data:
        return 1 if current_value > 0 else (-1 if current_value < 0 else 0)
    if not isinstance(previous_value, numbers.Number):
        return None
    change = current_value - previous_value
    return 1 if change > 0 else (-1 if change < 0 else 0)


def _numeric_vocab(vocab, device):
    key = (id(vocab), len(vocab), str(device))
    hit = _vocab_dev.get(key)
    if hit is not None:
        return hit
    numeric = all(isinstance(v, numbers.Number) for v in vocab)
    t = torch.tensor([float(v) for v in vocab], dtype=torch.float64, device=device) if numeric else None
    _vocab_dev[key] = (numeric, t)
    return numeric, t


def calculate_evaluation_metrics(logits_list, xb_list, yb_list, num_modalities, all_vocabularies, all_modality_params,
                                 all_file_info):
    """Per modality: (wins, losses, certainty_sum, batches_processed) of the last-token direction."""
    wins = [0] * num_modalities
    losses = [0] * num_modalities
    cert = [0.0] * num_modalities
    proc = [0] * num_modalities
    pending = []
    for i in range(num_modalities):
        if not (len(logits_list) > i and len(yb_list) > i):
            continue
        vocab = all_vocabularies[i]
        is_pct = bool(all_modality_params[i][3])
        lg = logits_list[i]
        numeric, vt = _numeric_vocab(vocab, lg.device)
        min_len = 1 if is_pct else 2
        if not (numeric and yb_list[i].ndim >= 2 and yb_list[i].shape[1] >= min_len):
            continue
        B, T, V = lg.shape
        if B == 0:
            continue
        if lg.device.type != "cuda":
            raise RuntimeError("calculate_evaluation_metrics runs on the GPU (mmt_eval_direction); no CPU path")
        proc[i] = 1
        acc_i = torch.zeros(2, dtype=torch.int32, device=lg.device)
        acc_c = torch.zeros(1, dtype=torch.float64, device=lg.device)
        xb = xb_list[i].contiguous()
        yb = yb_list[i].contiguous()
        lgc = lg.contiguous()
        rc = ML.lib().mmt_eval_direction(None, ML.stream_ptr(lg.device), B, T, V, ML.ptr(lgc), ML.ptr(xb),
                                         ML.ptr(yb), ML.ptr(vt), 1 if is_pct else 0, ML.ptr(acc_i), ML.ptr(acc_c))
        ML.check(rc, None, "mmt_eval_direction")
        pending.append((i, acc_i, acc_c, (lgc, xb, yb)))
    for i, acc_i, acc_c, _keep in pending:
        w, l = acc_i.tolist()
        wins[i], losses[i] = w, l
        cert[i] = float(acc_c.item())
    return wins, losses, cert, proc


# ------------------------------------------------------------------------------------------
# estimate_loss (reference training_utils.py:387-520)
# ------------------------------------------------------------------------------------------
def estimate_loss(current_step=None, max_steps=None):
    out = {}
    m.eval()
    for state in ["train", "val"]:
        now = datetime.now()
        current_time = now.strftime("%H:%M:%S")
        step_info = f"Step {current_step}/{max_steps} | " if current_step is not None else ""
        batch_calc = f" * {_get_batch_size()} batches = {_get_eval_iters() * _get_batch_size()} samples"
        print(f"Evaluation: {step_info}{state.title()} set ({_get_eval_iters()} iterations{batch_calc}) | {current_time}")
        tot_proc = [0] * num_modalities
        tot_ok = [0] * num_modalities
        tot_bad = [0] * num_modalities
        tot_cert = [0.0] * num_modalities
        loss_sum = None
        n_losses = 0
        with torch.no_grad():
            for k in range(_get_eval_iters()):
                xb_list, yb_list = get_batch(state, 0)
                logits_list, losses_list = m(xb_list, yb_list)
                if losses_list and all(l is not None for l in losses_list):
                    s = sum(losses_list)
                    loss_sum = s if loss_sum is None else loss_sum + s  # stays on device: one sync below
                    n_losses += 1
                else:
                    print(f"Warning: Iteration {k} losses not calculated, skipping")
                w, l, c, p = calculate_evaluation_metrics(logits_list, xb_list, yb_list, num_modalities,
                                                          all_vocabularies, all_modality_params, all_file_info)
                for i in range(num_modalities):
                    tot_ok[i] += w[i]
                    tot_bad[i] += l[i]
                    tot_cert[i] += c[i]
                    tot_proc[i] += p[i]
        out[state] = (loss_sum.item() / n_losses) if n_losses else float("nan")
        disp = "Train Set" if state == "train" else "Val Set"
        print(f"\nDIRECTIONAL METRICS - {disp} (Correct/Total)")
        for i in range(num_modalities):
            name = all_modality_params[i][9] if all_modality_params[i][9] else f"Modality {i+1}"
            if tot_proc[i] > 0:
                total = tot_ok[i] + tot_bad[i]
                if total > 0:
                    rate = round((tot_ok[i] / total) * 100, 1)
                    print(f"  - {name:<30}{tot_ok[i]}/{total} ({rate}%)")
                else:
                    print(f"  - {name}: No directional predictions")
            else:
                print(f"  - {name}: No data processed (non-numeric)")
        cfg = _get_config()
        output_file_name = cfg.get("output_file_name", "")
        project_file_path = cfg.get("project_file_path", "")
        if output_file_name != "":
            path = project_file_path + "output/" + output_file_name
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with open(path, "a", encoding="utf-8") as f:
                for i in range(num_modalities):
                    name = all_modality_params[i][9] if all_modality_params[i][9] else f"Modality {i+1}"
                    if tot_proc[i] > 0:
                        total = tot_ok[i] + tot_bad[i]
                        if total > 0:
                            rate = round((tot_ok[i] / total) * 100, 1)
                            f.write(f"   DIRECTIONAL PREDICTION {disp} - {name}: Correct={tot_ok[i]:,} | "
                                    f"Incorrect={tot_bad[i]:,} | Accuracy={rate}%\n")
                        else:
                            f.write(f"   DIRECTIONAL PREDICTION {disp} - {name}: Correct={tot_ok[i]:,} | "
                                    f"Incorrect={tot_bad[i]:,} | Accuracy=N/A\n")
                    else:
                        f.write(f"   DIRECTIONAL PREDICTION {disp} - {name}: Correct=0 | Incorrect=0 | Accuracy=N/A\n")
                if state == "train":
                    f.write("\n")
        if state == "train":
            print()
    m.train()
    sync_host_state()  # device-exact batcher: the host lists / Python random as the reference leaves them
    return out


# module globals injected by main.py (reference training_utils.py:523-534)
all_full_datasets = None
all_train_sets = None
all_val_sets = None
all_vocabularies = None
all_modality_params = None
all_file_info = None
file_lengths = None
num_modalities = None
is_percents = False
m = None
