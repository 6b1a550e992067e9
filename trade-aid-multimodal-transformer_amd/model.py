"""model.py — drop-in `MultimodalTransformer` backed by the gfx950 HIP library (libmmt_hip.so).

Same constructor, forward signature, state_dict keys/shapes and train()/eval() behaviour as the
reference (model.py:355-402 of tsnuk/trade-AId-multimodal-transformer):

    m = MultimodalTransformer(num_modalities, vocab_sizes, all_modality_params).to("cuda")
    logits_list, losses_list = m(idx_list, targets_list)
    sum(losses_list).backward()

Differences that are by design:
  * all parameters that receive gradients live in ONE flat fp32 `nn.Parameter` (`flat_params`);
    the parameters of a CrossAttention with no KV modality (M == 1, reference model.py:198-200,
    238), which never get a gradient, live in a second one (`flat_unused`) whose `.grad` stays
    None, so the reference's stock `torch.optim.AdamW(m.parameters(), lr)` (main.py:464) skips
    them exactly as it does in the reference. `state_dict()` / `load_state_dict()` expose and
    accept exactly the reference's per-head keys (including the `.tril` buffers, emitted as one
    shared tensor), so reference checkpoints round-trip;
  * compute runs in bf16 on MFMA with fp32 accumulation, fp32 master weights/residual stream;
  * forward/backward run only on a ROCm device (there is no CPU path: the CPU oracle lives in
    oracle/ and is test infrastructure only);
  * logits are outputs without autograd history (the reference training loop differentiates
    only the losses; main.py:646-649);
  * training batches are exactly block_size long (as the reference's get_batch makes them); a
    shorter sequence without targets (generate, inference) runs right-padded to block_size: the
    attention is causal, so the logits of the real positions are exactly those of the short run;
  * generate keeps a KV cache (one prefill forward, then one position per token through
    mmt_decode_step) while the sequence fits the block; the reference re-runs the forward.
"""
import ctypes

import torch
import torch.nn as nn

import mmt_lib as ML
from config_utils import _get_block_size, _get_dropout, _get_n_embd, _get_n_head, _get_n_layer, _get_precision


class _MmtStep(torch.autograd.Function):
    """One forward through the C-ABI; its backward is mmt_backward into a fresh flat grad."""

    @staticmethod
    def forward(ctx, flat, owner, training, n_mod, *tensors):
        idx = list(tensors[:n_mod])
        tgt = list(tensors[n_mod:]) if len(tensors) > n_mod else None
        logits, losses = owner._launch_forward(flat, idx, tgt, training)
        ctx.owner = owner
        ctx.gen = owner._gen
        ctx.keep = (idx, tgt)  # the engine reads the token ids again in the embedding backward
        ctx.n_tensors = len(tensors)
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(*logits)
        if losses is None:
            return tuple(logits)
        return (*logits, losses)

    @staticmethod
    def backward(ctx, *grads):
        g_losses = grads[-1]
        nones = (None,) * (3 + ctx.n_tensors)
        if g_losses is None:
            return nones
        owner = ctx.owner
        if owner._gen != ctx.gen:
            raise RuntimeError("MultimodalTransformer: backward of a stale forward (another forward ran in between); "
                               "the saved activations live in one workspace per model")
        grad = owner._launch_backward(g_losses)
        return (grad,) + nones


class MultimodalTransformer(nn.Module):
    """Reference model.py:355-402 (see module docstring)."""

    def __init__(self, num_modalities, vocab_sizes, all_modality_params):
        super().__init__()
        self.num_modalities = int(num_modalities)
        self.vocab_sizes = [int(v) for v in vocab_sizes]
        self.all_modality_params = all_modality_params
        M = self.num_modalities
        if not (1 <= M <= ML.MAX_MOD):
            raise ValueError("num_modalities must be 1..8")
        self.n_embd, self.n_head, self.n_layer = _get_n_embd(), _get_n_head(), _get_n_layer()
        self.block_size, self.dropout_p = _get_block_size(), float(_get_dropout())
        cfg = ML.MmtConfig()
        cfg.num_modalities = M
        cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.block_size = self.n_embd, self.n_head, self.n_layer, self.block_size
        for i in range(M):
            cfg.vocab_sizes[i] = self.vocab_sizes[i]
            cfg.cross_attention[i] = 1 if all_modality_params[i][8] else 0  # model.py:196
        cfg.dropout = self.dropout_p
        cfg.seed = 0
        self.precision = _get_precision()
        cfg.precision = 1 if self.precision == "fp8" else 0
        L = ML.lib()
        ctx = L.mmt_create(ctypes.byref(cfg))
        if not ctx:
            raise ML.MmtError("mmt_create failed: " + L.mmt_create_error().decode())
        self._ctx = ctypes.c_void_p(ctx)
        n = L.mmt_param_count(self._ctx)
        self._n_active = L.mmt_param_active_count(self._ctx)
        self._tensors = []
        name = ctypes.create_string_buffer(256)
        off, nd, shape, kind = ML.c_i64(), ML.c_i32(), (ML.c_i64 * 2)(), ML.c_i32()
        for i in range(L.mmt_tensor_count(self._ctx)):
            ML.check(L.mmt_tensor_info(self._ctx, i, name, 256, ctypes.byref(off), ctypes.byref(nd), shape,
                                       ctypes.byref(kind)), self._ctx, "mmt_tensor_info")
            shp = tuple(shape[d] for d in range(nd.value))
            self._tensors.append((name.value.decode(), off.value, shp, kind.value))
        self._tril_keys = self._make_tril_keys()
        flat = torch.zeros(n, dtype=torch.float32)
        self._init_flat(flat)
        na = self._n_active
        self.flat_params = nn.Parameter(flat[:na].clone())
        # never-used CrossAttention parameters (M == 1): their own Parameter, .grad stays None
        self.flat_unused = nn.Parameter(flat[na:].clone()) if n > na else None
        self._dropout_counter = 0
        self._dp_rank = 0  # data-parallel rank (mmt_dist.enable_data_parallel): folded into the dropout seed
        self._sticky_carry = 0  # sticky non-finite bits of workspaces replaced since the last clear
        self._ws = None
        self._ws_batch = -1
        self._ws_bytes = {}
        self._gen = 0
        self._last = None
        self._grad_sync = None  # mmt_dist.GradSync when data parallel

    # ------------------------------------------------------------------ layout / state_dict
    def _make_tril_keys(self):
        keys = []
        for l in range(self.n_layer):
            for i in range(self.num_modalities):
                for h in range(self.n_head):
                    keys.append(f"blocks.{l}.sa_layers.{i}.heads.{h}.tril")
            for i in range(self.num_modalities):
                if self.all_modality_params[i][8]:
                    for h in range(self.n_head):
                        keys.append(f"blocks.{l}.cross_attention_layers.{i}.heads.{h}.tril")
        return keys

    def _init_flat(self, flat):
        """model.py:372-378: Linear/Embedding weights N(0, 0.02), biases 0; LayerNorm 1 / 0."""
        for name, off, shp, kind in self._tensors:
            n = 1
            for s in shp:
                n *= s
            v = flat[off:off + n]
            if kind == 0:
                v.normal_(0.0, 0.02)
            elif kind == 2:
                v.fill_(1.0)
            else:
                v.zero_()

    def _view(self, off, shp, detach=False):
        """View of one reference tensor: a slice of flat_params, or of flat_unused past the
        active prefix."""
        n = 1
        for s in shp:
            n *= s
        if off >= self._n_active:
            base, off = self.flat_unused, off - self._n_active
        else:
            base = self.flat_params
        if detach:
            base = base.detach()
        return base[off:off + n].view(shp)

    def named_reference_tensors(self):
        """(reference state_dict key, view into flat_params) for every parameter."""
        for name, off, shp, _ in self._tensors:
            yield name, self._view(off, shp)

    def reference_grad_views(self):
        """(reference key, gradient view) for every parameter; None for the never-used ones."""
        g = self.flat_params.grad
        for name, off, shp, _ in self._tensors:
            if off >= self._n_active or g is None:
                yield name, None
                continue
            n = 1
            for s in shp:
                n *= s
            yield name, g[off:off + n].view(shp)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        for name, off, shp, _ in self._tensors:
            destination[prefix + name] = self._view(off, shp, detach=not keep_vars)
        if self._tril_keys:
            T = self.block_size
            tril = torch.tril(torch.ones(T, T, device=self.flat_params.device))
            for k in self._tril_keys:
                destination[prefix + k] = tril  # one shared storage (saved once by torch.save)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        known = set()
        with torch.no_grad():
            for name, off, shp, _ in self._tensors:
                key = prefix + name
                known.add(key)
                if key not in state_dict:
                    missing_keys.append(key)
                    continue
                src = state_dict[key]
                if tuple(src.shape) != tuple(shp):
                    error_msgs.append(f"size mismatch for {key}: copying a param with shape {tuple(src.shape)}, "
                                      f"the shape in current model is {tuple(shp)}.")
                    continue
                self._view(off, shp, detach=True).copy_(src)
        T = self.block_size
        for k in self._tril_keys:
            key = prefix + k
            known.add(key)
            if key not in state_dict:
                missing_keys.append(key)
            elif tuple(state_dict[key].shape) != (T, T):
                error_msgs.append(f"size mismatch for {key}: {tuple(state_dict[key].shape)} vs {(T, T)}")
        if strict:
            for key in state_dict.keys():
                if key.startswith(prefix) and key not in known:
                    unexpected_keys.append(key)
        self._gen += 1

    # ------------------------------------------------------------------ execution
    def _workspace(self, B, device):
        if B not in self._ws_bytes:
            self._ws_bytes[B] = ML.lib().mmt_workspace_bytes(self._ctx, B)
            if self._ws_bytes[B] < 0:
                raise ML.MmtError("mmt_workspace_bytes failed")
        if self._ws is None or self._ws_batch != B or self._ws.device != device:
            off = ML.lib().mmt_loss_flag_offset(self._ctx, B)  # the same offset for every batch size
            if self._ws is not None:  # keep the sticky bits of the workspace being replaced
                self._sticky_carry |= int(self._ws[off + 4:off + 8].view(torch.int32).item())
            self._ws = None
            self._ws = torch.empty(self._ws_bytes[B], dtype=torch.uint8, device=device)
            self._ws_batch = B
            self._ws[off:off + 8].zero_()  # non-finite-loss flags (last forward, sticky)
        return self._ws

    def _launch_forward(self, flat, idx, tgt, training):
        L = ML.lib()
        dev = flat.device
        B, T = idx[0].shape
        ws = self._workspace(B, dev)
        logits = [torch.empty(B, T, V, dtype=torch.float32, device=dev) for V in self.vocab_sizes]
        losses = torch.empty(self.num_modalities, dtype=torch.float32, device=dev) if tgt is not None else None
        idx_arr = ML.ptr_array(idx)
        tgt_arr = ML.ptr_array(tgt) if tgt is not None else None
        if training:
            self.last_dropout_seed = self._next_dropout_seed(dev)
            ML.check(L.mmt_set_dropout_seed(self._ctx, self.last_dropout_seed), self._ctx, "mmt_set_dropout_seed")
        with torch.cuda.device(dev):
            rc = L.mmt_forward(self._ctx, ML.stream_ptr(dev), B, idx_arr, tgt_arr, ML.ptr(flat), ML.ptr_array(logits),
                               ML.ptr(losses), ML.ptr(ws), 1 if training else 0)
        ML.check(rc, self._ctx, "mmt_forward")
        self._gen += 1
        self._last = (flat, idx, tgt)
        return logits, losses

    def _next_dropout_seed(self, dev):
        """Seed of this training step's dropout masks. The reference's nn.Dropout on a ROCm device
        draws from the device generator, never from torch's CPU generator (which get_batch's
        torch.randint start indices consume), so the seed is derived from the device generator's
        seed and Philox offset and the CPU random stream stays the reference's. The offset is
        bumped by a fixed 4 per forward only to keep the seed sequence repeatable under
        torch.manual_seed; this does NOT reproduce the reference's Philox consumption (its dropout
        calls advance the offset by tensor size), so later device-RNG users (e.g.
        torch.multinomial in generate) see a different stream than the reference's. Under data
        parallelism the rank is folded in: each rank draws its own masks."""
        self._dropout_counter += 1
        seed, off = 0, self._dropout_counter
        try:
            gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
            seed = int(gen.initial_seed())
            off = int(gen.get_offset())
            gen.set_offset(off + 4)
        except (AttributeError, RuntimeError, IndexError):
            pass
        x = (seed * 0x9E3779B97F4A7C15 + off * 0xBF58476D1CE4E5B9 + self._dropout_counter
             + self._dp_rank * 0xD1B54A32D192ED03) & (2 ** 64 - 1)
        x ^= x >> 31
        x = (x * 0x94D049BB133111EB) & (2 ** 64 - 1)
        return int(x ^ (x >> 29)) & (2 ** 62 - 1)

    def nonfinite_loss_mask(self, sticky=False, clear=False):
        """Device int32 bitmask, bit i set when modality i's loss was NaN / Inf (set by the loss
        kernel): of the last forward with targets, or (sticky=True) of every
        forward since the sticky word was last cleared (clear=True clears it). A copy, no sync."""
        if self._ws is None:
            return None
        off = ML.lib().mmt_loss_flag_offset(self._ctx, self._ws_batch) + (4 if sticky else 0)
        w = self._ws[off:off + 4]
        out = w.view(torch.int32).clone()
        if sticky and self._sticky_carry:
            out |= self._sticky_carry
        if clear:
            w.zero_()
            if sticky:
                self._sticky_carry = 0
        return out

    def backward_stage_ranges(self):
        """[(begin, end)] of the flat gradient finalised by each backward stage, in execution order
        (post block, layers L-1..0, embeddings); see mmt_backward_stage_range in include/mmt.h."""
        L = ML.lib()
        out = []
        b, e = ML.c_i64(), ML.c_i64()
        for s in range(L.mmt_backward_stage_count(self._ctx)):
            ML.check(L.mmt_backward_stage_range(self._ctx, s, ctypes.byref(b), ctypes.byref(e)), self._ctx,
                     "mmt_backward_stage_range")
            out.append((b.value, e.value))
        return out

    def _launch_backward(self, g_losses):
        L = ML.lib()
        flat = self._last[0]
        g = g_losses.detach().to(dtype=torch.float32).contiguous()
        grad = torch.empty_like(flat)
        sync = self._grad_sync
        with torch.cuda.device(flat.device):
            if sync is None:
                rc = L.mmt_backward(self._ctx, ML.stream_ptr(flat.device), ML.ptr(g), ML.ptr(flat), ML.ptr(grad),
                                    ML.ptr(self._ws))
                ML.check(rc, self._ctx, "mmt_backward")
                return grad
            # data parallel (mmt_dist): stage by stage, each finished bucket all-reduced while the
            # next stages compute
            for s in range(L.mmt_backward_stage_count(self._ctx)):
                rc = L.mmt_backward_stage(self._ctx, ML.stream_ptr(flat.device), s, ML.ptr(g), ML.ptr(flat),
                                          ML.ptr(grad), ML.ptr(self._ws))
                ML.check(rc, self._ctx, "mmt_backward_stage")
                sync.stage_done(s, grad)
            sync.finish()
        return grad

    def forward(self, idx_list, targets_list=None):
        """model.py:380-402: returns (logits_list, losses_list | None)."""
        M = self.num_modalities
        if len(idx_list) != M:
            raise ValueError(f"expected {M} index tensors, got {len(idx_list)}")
        flat = self.flat_params
        if flat.device.type != "cuda":
            raise RuntimeError("MultimodalTransformer (libmmt_hip) runs only on a ROCm GPU: call .to('cuda') "
                               "(there is no CPU path)")
        B, T = idx_list[0].shape
        if T > self.block_size:
            raise ValueError(f"sequence length {T} exceeds block_size {self.block_size}")
        if T < self.block_size and targets_list is not None:
            raise NotImplementedError(f"training on sequence length {T} < block_size {self.block_size}: the training "
                                      f"batches of the reference are always block_size long")
        idx = [t.to(device=flat.device, dtype=torch.long).contiguous() for t in idx_list]
        for t in idx:
            if tuple(t.shape) != (B, T):
                raise ValueError("all modalities must share the [B, T] batch shape")
        if T < self.block_size:
            # causal: position t sees tokens <= t only, so right padding leaves positions < T unchanged
            pad = self.block_size - T
            idx = [torch.nn.functional.pad(t, (0, pad)) for t in idx]
            logits = _MmtStep.apply(flat, self, False, M, *idx)
            return [lg[:, :T] for lg in logits], None
        tensors = list(idx)
        if targets_list is not None:
            tensors += [t.to(device=flat.device, dtype=torch.long).contiguous() for t in targets_list]
        training = bool(self.training and self.dropout_p > 0.0)
        outs = _MmtStep.apply(flat, self, training, M, *tensors)
        logits = list(outs[:M])
        if targets_list is None:
            return logits, None
        losses = outs[M]
        return logits, [losses[i] for i in range(M)]

    @torch.no_grad()
    def generate(self, idx_list, max_new_tokens=1, modality_to_generate=0, use_cache=True, sample_fn=None):
        """model.py:404-446: per new token, the logits of the last position of the (block_size
        cropped) context, a sample from the softmax of the target modality's last logits
        (torch.multinomial, as the reference; `sample_fn(probs) -> [B, 1]` overrides it), appended;
        the other modalities are padded with their last token or cropped to the same length.

        The reference re-runs the whole forward per token. Here, while the sequence still fits the
        block (positions do not shift), the first step is one forward over the prompt (the prefill,
        which leaves the keys / values of every position in the workspace) and every later step is
        ONE position through the KV-cache decode of the engine (mmt_decode_step): the same logits
        (causal attention, absolute positions) at O(t) instead of O(block_size) attention and no
        re-run of the prompt's GEMMs. Once the sequence outgrows the block every position shifts
        and it falls back to the reference's full re-forward. use_cache=False (or training mode
        with dropout, where the reference's forward samples dropout, or the fp8 precision, whose
        forward GEMMs the bf16 decode would not reproduce) always re-runs the forward."""
        seqs = [idx.clone() for idx in idx_list]
        T = self.block_size
        g = modality_to_generate
        sample = sample_fn or (lambda probs: torch.multinomial(probs, num_samples=1))
        cache = (use_cache and not (self.training and self.dropout_p > 0.0) and self.precision == "bf16"
                 and len({int(s.shape[1]) for s in seqs}) == 1 and all(s.dim() == 2 for s in seqs))
        cached_pos = None  # the last position whose keys / values the workspace holds
        for _ in range(max_new_tokens):
            n = seqs[g].shape[1]
            if cache and cached_pos is not None and n - 1 == cached_pos + 1 and n <= T:
                last = self._decode_step([s[:, n - 1] for s in seqs], n - 1)[g]
                cached_pos = n - 1
            else:
                cond = [s[:, -T:] for s in seqs]
                logits, _ = self(cond)
                last = logits[g][:, -1, :]
                cached_pos = n - 1 if (cache and n <= T) else None
            probs = torch.softmax(last, dim=-1)
            nxt = sample(probs).to(seqs[g].dtype)
            seqs[g] = torch.cat((seqs[g].to(nxt.device), nxt), dim=1)
            n = seqs[g].shape[1]
            for i in range(self.num_modalities):
                if i == g:
                    continue
                if seqs[i].shape[1] < n:
                    seqs[i] = torch.cat((seqs[i], seqs[i][:, -1:]), dim=1)
                elif seqs[i].shape[1] > n:
                    seqs[i] = seqs[i][:, :n]
        return seqs

    @torch.no_grad()
    def _decode_step(self, tokens, pos):
        """Logits [B, V_i] of every modality at position `pos` (1 <= pos < block_size), given the
        tokens [B] of that position; the workspace must hold positions < pos (a forward over them,
        then decode steps; include/mmt.h mmt_decode_step)."""
        flat = self.flat_params
        dev = flat.device
        B = tokens[0].shape[0]
        if self._ws is None or self._ws_batch != B:
            raise RuntimeError("_decode_step: no prefill forward at this batch size")
        idx = [t.to(device=dev, dtype=torch.long).contiguous() for t in tokens]
        logits = [torch.empty(B, V, dtype=torch.float32, device=dev) for V in self.vocab_sizes]
        L = ML.lib()
        with torch.cuda.device(dev):
            rc = L.mmt_decode_step(self._ctx, ML.stream_ptr(dev), B, int(pos), ML.ptr_array(idx), ML.ptr(flat),
                                   ML.ptr_array(logits), ML.ptr(self._ws))
        ML.check(rc, self._ctx, "mmt_decode_step")
        self._gen += 1
        self._keep_decode = idx  # alive until the step's kernels have read them
        return logits

    def __del__(self):
        try:
            if getattr(self, "_ctx", None):
                ML.lib().mmt_destroy(self._ctx)
                self._ctx = None
        except Exception:
            pass
