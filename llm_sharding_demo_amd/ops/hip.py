"""HIP backend: the engine ops on the hand-written gfx950 kernels (_C.so).

There is no fallback: constructing `HipBackend` without the built extension
raises, so a GPU run can never silently execute eager PyTorch math.

Device weight layout (set up once per stage by `prepare_stage`):
  * lm_head rows padded to a multiple of 64 (50257 -> 50304) so the logits
    GEMM tiles evenly; padded logits are never sampled (sampler scans < V).
  * Llama q/k projection rows re-ordered per head so RoPE pairs (i, i+hd/2)
    become adjacent columns (2i, 2i+1): the QKV epilogue then rotates with one
    lane exchange.  Q.K is invariant to a common permutation of head dims, so
    q and the K cache simply live in that order.
  * Llama gate/up rows interleaved in 16-row blocks so one wave holds the gate
    and up value of the same output column (silu(gate)*up fused epilogue).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import Backend, Residual

_C = None
_ERR: Optional[BaseException] = None


def _load():
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        from .. import _C as ext  # built in-tree by ops/build.py
    except ImportError as e:  # pragma: no cover
        _ERR = e
        raise RuntimeError(
            "llm_sharding_demo_amd._C (the gfx950 HIP kernels) is not built or failed to load; "
            "run `python -m llm_sharding_demo_amd.ops.build` (or __graft_entry__.build())") from e
    _C = ext
    return _C


def extension_loaded() -> bool:
    try:
        _load()
        return True
    except Exception:
        return False


def rope_pair_permutation(n_heads: int, hd: int) -> torch.Tensor:
    half = hd // 2
    per = []
    for i in range(half):
        per += [i, i + half]
    idx = torch.tensor(per)
    return torch.cat([h * hd + idx for h in range(n_heads)])


def interleave_gate_up(w: torch.Tensor, f: int, blk: int = 16) -> torch.Tensor:
    gate, up = w[:f], w[f:]
    h = w.shape[1]
    return torch.stack([gate.reshape(f // blk, blk, h), up.reshape(f // blk, blk, h)], 1).reshape(2 * f, h)


def rope_table(max_pos: int, hd: int, theta: float, device) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], -1).float().contiguous().to(device)


def prefill_tiles(meta) -> torch.Tensor:
    """(sequence, query offset) of every 64-query tile of a packed batch."""
    qlens = meta.host_qlens
    tiles = [(i, off) for i, n in enumerate(qlens) for off in range(0, n, 64)]
    return torch.tensor(tiles, dtype=torch.int32).reshape(-1, 2)


class LazyNorm:
    """A norm whose output has not been materialised: at M <= GEMV_NORM_MAX_M
    rows the consuming GEMV (csrc/kernels/gemv.hip) normalises the fp32
    residual rows itself, so the separate norm launch disappears.  Any other
    consumer materialises it through the norm kernel."""

    __slots__ = ("x", "w", "b", "eps", "rms")

    def __init__(self, x, w, b, eps, rms):
        self.x, self.w, self.b, self.eps, self.rms = x, w, b, eps, rms

    @property
    def shape(self):
        return self.x.shape

    @property
    def code(self) -> int:  # gemv norm code: 1 LayerNorm, 2 RMSNorm
        return 2 if self.rms else 1


# gemv epilogue codes (csrc/kernels/gemm.hip Epi)
_EPI = {"none": 0, "gelu": 1, "silu_mul": 2}
EPI_F32, EPI_RESID, EPI_QKV = 3, 4, 6


class HipBackend(Backend):
    name = "hip"
    # Decode GEMMs of at most GEMV_MAX_M rows run on the weight-streaming GEMV
    # (no split-K, fused epilogues); at most GEMV_NORM_MAX_M rows it also folds
    # the preceding LayerNorm / RMSNorm into its prologue.  0 disables.
    GEMV_MAX_M = int(os.environ.get("LSD_GEMV_MAX_M", "8"))
    GEMV_NORM_MAX_M = int(os.environ.get("LSD_GEMV_NORM_MAX_M", "2"))
    TARGET_BLOCKS = 512  # >> 256 CUs so every CU streams
    # Grouped-query decode attention on MFMA (attention.hip
    # attn_decode_mfma_kernel, one wave per (sequence, kv head, split)): taken
    # at >= ATTN_MFMA_MIN waves (the kernel's own default).  Fewer than
    # ATTN_MFMA_SPLIT_BELOW items (long contexts, few sequences) split the
    # context towards ATTN_MFMA_WAVES waves, >= 512 keys per split.  1024
    # waves measured best (Llama-3 8B shapes, 2K-8K contexts: 1.3-1.45x the
    # split VALU kernel; profiles/r2_long_context.log)
    ATTN_MFMA_MIN = 256
    ATTN_MFMA_SPLIT_BELOW = 1024
    ATTN_MFMA_WAVES = int(os.environ.get("LSD_ATTN_MFMA_WAVES", "1024"))
    # decode GEMM: aim for this many workgroups (column tiles x k-splits)
    # decode (split-K, last-arriver) GEMM up to this many rows (above 128 as
    # row blocks of <= 128 sharing each W tile); tiled above.  256-row decode
    # microbatches: 41.2k vs 39.7k tok/s on the tiled kernel (GPT-2 XL, 2 x 256)
    SK_MAX_M = int(os.environ.get("LSD_SK_MAX_M", "256"))
    DEFER_RESID = os.environ.get("LSD_DEFER_RESID", "1") == "1"
    # prefill residual projections as one bf16 slab folded by the next norm
    # instead of the GEMM epilogue's fp32 read-modify-write of the residual:
    # prefill 222.6 / 225.1 vs 224.5 / 225.8 ms on the headline, within noise
    # (profiles/r5_prefill_slab_ab.log) -- opt-in (LSD_PREFILL_SLAB=1)
    PREFILL_SLAB = os.environ.get("LSD_PREFILL_SLAB", "0") == "1"
    # prefill GEMMs hipBLASLt runs with its own fused epilogues (csrc/blaslt.cpp),
    # where it measured faster than the hand-written 256x256 kernel
    # (profiles/r5_blaslt.log): residual projections (x += a w^T + b, fp32 x)
    # with K >= BLASLT_RESID_MIN_K (GPT-2 XL proj2 +5 %, Llama-3 8B o / down
    # +6 %; K 1600 loses 12 % at 32 K rows) and MLP-up bias + GELU from
    # BLASLT_GELU_MIN_M rows (+11 % at 64 K rows, a tie at 32 K).  Only at or
    # above BLASLT_MIN_M rows (0 = never).
    BLASLT_MIN_M = int(os.environ.get("LSD_BLASLT_MIN_M", "4096"))
    BLASLT_RESID_MIN_K = int(os.environ.get("LSD_BLASLT_RESID_MIN_K", "4096"))
    BLASLT_GELU_MIN_M = int(os.environ.get("LSD_BLASLT_GELU_MIN_M", "65536"))
    # decode gate_up (SiLU * up) at BLASLT_SILU_MIN_M..MAX_M rows: the hipBLASLt
    # GEMM, then the elementwise pass (elementwise.hip).  Llama-3 8B bench
    # (profiles/r5_llama_blaslt.log): 128 rows +1.7 % (18.15 / 18.12k vs 17.84k
    # tok/s), 256 rows -1.2 %, 512 rows -1 to -1.5 % although faster alone
    # there (132 -> 109 + ~8 us, tools/bench_llama_blaslt.py): on for 64-128
    # rows.  MIN 0 = off
    BLASLT_SILU_MIN_M = int(os.environ.get("LSD_BLASLT_SILU_MIN_M", "64"))
    # decode MLP-up (bias + GELU) on hipBLASLt from this many rows: GPT-2 XL at
    # 384 / 512 rows 24.6 / 25.3 -> 21.3 / 22.6 us alone; 1024 sequences
    # (2 x 512) 56.2k -> 56.7k tok/s, p50 14.95 -> 14.68 ms
    # (profiles/r5_xl_decode_gelu.log).  Below 384 rows the ring kernels win
    # (profiles/r5_small_k_routing.log).  0 = off
    BLASLT_DECODE_GELU_MIN_M = int(os.environ.get("LSD_BLASLT_DECODE_GELU_MIN_M", "384"))
    BLASLT_SILU_MAX_M = int(os.environ.get("LSD_BLASLT_SILU_MAX_M", "128"))
    # decode QKV from this many rows with K >= BLASLT_QKV_MIN_K on hipBLASLt
    # (fp32 out) + the RoPE / cache-append pass (elementwise.hip qkv_post):
    # Llama-3 8B at 512 rows 52.5 us on the 8-wave ring vs 38.6 us for the
    # library GEMM alone (profiles/r5_llama_blaslt.log).  0 = off
    BLASLT_QKV_MIN_M = int(os.environ.get("LSD_BLASLT_QKV_MIN_M", "512"))
    BLASLT_QKV_MIN_K = int(os.environ.get("LSD_BLASLT_QKV_MIN_K", "4096"))
    # Decode GEMM workgroup target (column tiles x K splits).  With c microbatch
    # lanes running concurrently each GEMM should fill ~1/c of the chip so the
    # lanes' kernels co-reside: 384 alone, 192 with two lanes (bench sweep:
    # 31.1k -> 32.1k tok/s, GPT-2 XL, 2 x 128 rows).  LSD_SK_TARGET overrides.
    SK_TARGET = int(os.environ.get("LSD_SK_TARGET", "0")) or None
    SK_MIN_STEPS = int(os.environ.get("LSD_SK_MIN_STEPS", "2"))  # 32-k steps per split
    # decode GEMM rows per row block when an under-filled grid (deferred
    # residual projections) is split into row blocks (sk_rblocks in gemm.hip)
    SK_ROWS = int(os.environ.get("LSD_SK_ROWS", "64"))
    # decode GEMM 128-column tiles above this many rows (off: slower, see gemm.hip)
    NW2_ROWS = int(os.environ.get("LSD_NW2_ROWS", str(1 << 30)))
    # tiled launches of at most this many workgroups run the LDS ring variant
    # (steps kt+1, kt+2 in flight while kt computes; 1 block/CU); 0 = off.  At
    # 256 rows and 128x128 tiles QKV 25.8 -> 20.4 us, MLP-up 29.6 -> 23.3;
    # lm_head's 393-tile grid at 128 rows is better on the 2-blocks/CU kernel
    # (45.2 vs 47.7 us); 4 slots = 3 slots (profiles/r1_ab_ring_n64.log)
    # Counted in 128x64 tiles (a 128x128 ring grid may use half).  512:
    # Llama-3 8B's 28672-wide gate/up at 128 rows (448 tiles of 128x64) joins
    # the ring, 18.6k -> 18.9k tok/s; residual splits keep their own 256
    # target (RING_RESID_TARGET: GPT-2 XL loses 7 % with 512-WG slabs)
    TILED3_MAX = int(os.environ.get("LSD_TILED3_MAX", "512"))
    RING_SLOTS = int(os.environ.get("LSD_RING_SLOTS", "3"))  # 3 or 4 (128 KiB of LDS)
    # ring tile columns, 128 or 64.  128x64 tiles double the workgroups of the
    # decode-sized grids: at 256 rows QKV 20.5 -> 15.6 us, MLP-up 23.5 -> 17.3
    # (split-K kernel 23.3 / 26.2, hipBLASLt 19.3 / 20.0); bench 42.9k -> 43.8k
    RING_TN = int(os.environ.get("LSD_RING_TN", "0"))
    # auto (RING_TN = 0): 128x32 ring tiles (2 blocks/CU) when the 128x64 grid
    # has fewer workgroups than this -- 128 rows: QKV 15.9 -> 13.2 us, MLP-up
    # 17.2 -> 14.2; at 256 rows the 64-wide tiles stay faster (15.6 vs 18.6)
    # (profiles/r2_ring_tn32.log)
    RING_FILL = int(os.environ.get("LSD_RING_FILL", "128"))
    # above 128 rows: 96-row ring tiles when 3 x the 64-wide column tiles are at
    # most this many workgroups (0 = off, default: faster alone, slower beside
    # the other lane; gemm.hip, profiles/r2_ring_m96.log); unsplit GEMMs only
    RING_M96 = int(os.environ.get("LSD_RING_M96", "0"))
    # Decode GEMMs leave split-K for the tiled kernels (the 128x64 LDS ring at
    # these grid sizes) above TILED_ALL_M rows at any width, and above
    # TILED_MIN_M rows when at least TILED_MIN_N wide.  bench tok/s (1 MI355X,
    # profiles/r1_ab_tiled_min_n.log, r1_ab_ring_n64.log):
    #   GPT-2 XL 2 x 256: split-K 41.2-41.6k; MLP-up + QKV tiled 43.8k; all 46.3-46.6k
    #   GPT-2 small 2 x 256: split-K 286.8k; all tiled 309.8k
    #   GPT-2 XL 2 x 128: split-K 34.0k; all tiled 33.3k (N = 1600 prefers split-K at 128 rows)
    #   Llama-3 8B 2 x 128: split-K 17.0k; >= 4800 wide 18.0-18.2k; all (N >= 4096) 18.7k
    TILED_ALL_M = int(os.environ.get("LSD_TILED_ALL_M", "128"))
    # workgroup target of split-K residual GEMMs on the ring (0 = TILED3_MAX)
    RING_RESID_TARGET = int(os.environ.get("LSD_RING_RESID_TARGET", "256"))
    # 128x128-tile target of residual projections for decode groups of
    # 257-1024 rows (0 = the prefill rule, ~256 tiles); see _resid_splits
    RESID_WG_TARGET = int(os.environ.get("LSD_RESID_WG_TARGET", "1024"))
    # 8 K splits for K >= 8192 residual projections of 129-256 rows (0 = off)
    RESID_LONGK = int(os.environ.get("LSD_RESID_LONGK", "1"))
    RESID_LONGK_MIN_M = int(os.environ.get("LSD_RESID_LONGK_MIN_M", "128"))
    TILED_MIN_M = int(os.environ.get("LSD_TILED_MIN_M", "64"))
    # Decode GEMMs of 129-256 rows on the 8-wave all-rows kernel (gemm.hip
    # gemm_d256_kernel): 1 = auto (long-K GEMMs, below), 64 / 128 = every
    # 129-256-row tiled GEMM with that tile width (A/B), 0 = off (the 128x64
    # ring).  Ring depth, and the workgroup targets that set the K splits of
    # the in-kernel-combined GEMMs (QKV, MLP-up) and of the residual slabs.
    # Auto (tools/bench_d256.py at 256 rows, profiles/r3_d256_ab.log): Llama-3
    # 8B gate/up 84.6 -> 69.0 us (128-wide tiles, 224 workgroups, no split),
    # QKV 35.6 -> 31.9 (64-wide, 2 K splits); GPT-2 XL's K = 1600 GEMMs stay on
    # the ring (16.6 vs 16.9-20.6 us; bench 49.0k vs 45.2-47.1k tok/s)
    D256 = int(os.environ.get("LSD_D256", "1"))
    D256_MIN_K = int(os.environ.get("LSD_D256_MIN_K", "4096"))
    D256_SLOTS = int(os.environ.get("LSD_D256_SLOTS", "3"))
    D256_TARGET = int(os.environ.get("LSD_D256_TARGET", "192"))
    D256_RESID_TARGET = int(os.environ.get("LSD_D256_RESID_TARGET", "192"))
    D256_RESID = int(os.environ.get("LSD_D256_RESID", "0"))  # residual projections too
    TILED_MIN_N = int(os.environ.get("LSD_TILED_MIN_N", "4000"))
    # 128x64 decode ring on 8 waves (gemm.hip gemm_ring8_kernel): 0 = the
    # 4-wave ring, 1 = 4 computing + 4 loader waves, 2 = 8 computing waves.
    # 256 rows (tools/bench_d256.py, profiles/r3_ring8_ab.log): GPT-2 XL QKV
    # 16.7 -> 15.2 us, MLP-up 17.5 -> 15.8, residual projections 3-6 %
    # faster; bench 48.9k -> 49.7k tok/s (p50 8.54 -> 8.38 ms).  A 4-slot
    # ring is faster alone (QKV 14.4 us) but slower beside the other lane
    # (p50 8.72 ms: 96 KiB of LDS per workgroup), so 3 slots.
    RING8 = int(os.environ.get("LSD_RING8", "2"))
    RING8_FLAGS = int(os.environ.get("LSD_RING8_FLAGS", "0"))  # A/B bits (gemm.hip)
    # norms of at least this many rows run one wave per row (norm.hip
    # norm_wave_kernel): prefill 32 K rows x 1600 97.7 -> 53.7 us, x 768 71.5
    # -> 24.4 us, x 4096 a tie; GPT-2 XL prefill 217 -> 210 ms
    # (profiles/r5_normwave.log).  0 = the block-per-row kernel everywhere
    NORM_WAVE_MIN = int(os.environ.get("LSD_NORM_WAVE_MIN", "4096"))
    # ... and from this many rows when H <= 1024, with or without split-K
    # slabs to fold: GPT-2 small decode at 2 x 256 rows 351.1-351.3k ->
    # 354.2-355.0k tok/s (profiles/r5_normwave_decode.log).  GPT-2 XL's H =
    # 1600 decode norms lost 1.6 % on it and keep the block kernel
    # (profiles/r5_normwave_slab.log).  The choice depends on (rows, H) only,
    # so a pipeline stage boundary (slabs folded before the norm) computes the
    # same statistics as one stage; 0 = off
    NORM_WAVE_NARROW_MIN = int(os.environ.get("LSD_NORM_WAVE_NARROW_MIN", "256"))
    # lm_head epilogue writes 8-logit segment maxima for the sampler (sample.hip)
    SEGMAX = int(os.environ.get("LSD_SEGMAX", "1"))
    # K splits of the non-residual decode GEMMs on the 8-wave ring (QKV, MLP-up,
    # 129-256 rows) with the in-kernel last-arriver combine: aim at this many
    # workgroups (0 = off: one workgroup per 128x64 tile)
    RING8_SK_TARGET = int(os.environ.get("LSD_RING8_SK_TARGET", "0"))

    def __init__(self):
        self.C = _load()
        self.C.gemm_set_sk_rows(self.SK_ROWS)
        self.C.gemm_set_nw2_rows(self.NW2_ROWS)
        self.C.gemm_set_tiled3_max(self.TILED3_MAX)
        self.C.gemm_set_ring_slots(self.RING_SLOTS)
        self.C.gemm_set_ring_tn(self.RING_TN)
        self.C.gemm_set_ring_fill(self.RING_FILL)
        self.C.gemm_set_ring_m96(self.RING_M96)
        self.C.gemm_set_d256_slots(self.D256_SLOTS)
        self.C.gemm_set_ring8(self.RING8)
        self.C.gemm_set_ring8_flags(self.RING8_FLAGS)
        self.C.norm_set_wave_min(self.NORM_WAVE_MIN)
        self.C.norm_set_wave_narrow_min(self.NORM_WAVE_NARROW_MIN)
        self.C.attn_set_max_wg(int(os.environ.get("LSD_ATTN_MAX_WG", "0")))
        self.C.gemv_set_nt(int(os.environ.get("LSD_GEMV_NT", "0")))
        self.C.attn_set_small_waves(int(os.environ.get("LSD_ATTN_SMALL_WAVES", "8")))
        lw = int(os.environ.get("LSD_ATTN_LARGE_WAVES", "4"))  # full-batch decode attention block (4 / 8 waves)
        self.C.attn_set_large_waves(64, lw)
        self.C.attn_set_large_waves(128, lw)
        self.counters = None
        self._rope = None
        self.lane = 0  # microbatch lane (stream) currently being issued; see pipeline.py
        self.concurrency = 1  # microbatch lanes running at once (set per round by the pipeline)

    # ------------------------------------------------------------------
    def prepare_stage(self, stage) -> None:
        cfg, w, dev = stage.cfg, stage.w, stage.device
        if stage.last:
            # pad the head IN PLACE: the stage keeps one [vocab_padded, H]
            # tensor and its weight dict points at the first V rows (a
            # contiguous view -- the tied GPT-2 embedding of a 1-stage pipeline
            # reads the same rows), so the unpadded copy is freed
            key = "wte" if cfg.arch == "gpt2" else "lm_head"
            head = w[key]
            if head.shape[0] == cfg.vocab_padded:
                stage._lm_head_padded = head
            else:
                pad = torch.zeros(cfg.vocab_padded, cfg.hidden, dtype=head.dtype, device=dev)
                pad[: cfg.vocab_size] = head
                w[key] = pad[: cfg.vocab_size]
                del head
                stage._lm_head_padded = pad
        if cfg.arch == "llama":
            perm_q = rope_pair_permutation(cfg.n_heads, cfg.head_dim)
            perm_k = rope_pair_permutation(cfg.n_kv_heads, cfg.head_dim) + cfg.q_size
            keep = torch.arange(cfg.q_size + cfg.kv_size, cfg.qkv_size)
            perm = torch.cat([perm_q, perm_k, keep]).to(dev)
            for i in stage.layers:  # a boundary layer may hold only one half here
                p = f"layers.{i}."
                if p + "self_attn.qkv.weight" in w:
                    w[p + "self_attn.qkv.weight"] = w[p + "self_attn.qkv.weight"].index_select(0, perm).contiguous()
                if p + "mlp.gate_up.weight" in w:
                    w[p + "mlp.gate_up.weight"] = interleave_gate_up(w[p + "mlp.gate_up.weight"], cfg.ffn).contiguous()
            stage._rope = rope_table(stage.max_seq, cfg.head_dim, cfg.rope_theta, dev)
        else:
            stage._rope = None
        self._rope = getattr(stage, "_rope", None)
        # split-K ticket counters: zero at rest, re-armed by each tile's last
        # arriver; one row per microbatch lane so concurrent lanes never share one
        self._counters = torch.zeros(8, 1 << 16, dtype=torch.int32, device=dev)
        stage._hip_prepared = True

    @property
    def counters(self):
        return None if self._counters is None else self._counters[self.lane % 8]

    @counters.setter
    def counters(self, value):
        self._counters = None if value is None else value.reshape(-1, 1 << 16)

    # ------------------------------------------------------------------
    @classmethod
    def _tiled(cls, M: int, N: int = 0) -> bool:
        return (M > cls.SK_MAX_M or M > cls.TILED_ALL_M
                or (M > cls.TILED_MIN_M and N >= cls.TILED_MIN_N))

    def _d256_bn(self, M: int, N: int, K: int) -> int:
        """Tile columns when this GEMM runs on gemm_d256_kernel, else 0
        (mirrors d256_bn() in gemm.hip)."""
        if not self.D256 or not (128 < M <= 256) or K % 64 or N > 32768 or not self._tiled(M, N):
            return 0
        if self.D256 == 1:  # auto: long-K GEMMs only; 128-wide tiles when they alone fill the chip
            if K < self.D256_MIN_K:
                return 0
            return 128 if N % 128 == 0 and N // 128 >= 128 else 64
        return 128 if self.D256 == 128 and N % 128 == 0 else 64

    @staticmethod
    def _d256_kind(bn: int) -> int:  # lsd_gemm launch kind of gemm_d256
        return 3 if bn == 128 else 2

    def _d256_splits(self, N: int, K: int, bn: int, target: int) -> int:
        tiles = math.ceil(N / bn)
        return max(1, min(round(target / tiles), K // 64 // 2 or 1, 16))

    def _resid_splits(self, M: int, N: int, K: int) -> int:
        bn = self._d256_bn(M, N, K)
        if bn and self.D256_RESID:
            return self._d256_splits(N, K, bn, self.D256_RESID_TARGET)
        if self._tiled(M, N):
            if M <= self.SK_MAX_M and self.TILED3_MAX and self.RING_TN in (0, 32, 64):
                # decode rows on the 128x64 ring: as many splits as keep the
                # grid on the ring kernel
                # at most one split per 512 of K: short-K projections lose more
                # to the slab combine than they gain in workgroups (GPT-2 XL
                # attention out-proj, K = 1600: 3 splits 11.8 us vs 5 splits
                # 12.6 at 256 rows, 9.2 vs 9.3 at 128; profiles/r2_ring_tn32.log)
                if M > self.RESID_LONGK_MIN_M and K >= 8192 and self.RESID_LONGK:
                    # long-K projections above 128 rows: 8 splits, which leaves
                    # the ring for the 128x128 tiled kernel -- Llama-3 8B down at
                    # 256 rows 71.9 -> 55.3 us with its norm (2 ring splits);
                    # profiles/r2_resid512_splits.log
                    return min(8, K // 1024)
                tiles = math.ceil(M / 128) * math.ceil(N / 64)
                target = min(self.TILED3_MAX, self.RING_RESID_TARGET or self.TILED3_MAX)
                return max(1, min(target // tiles, K // 512 or 1))
            tiles = math.ceil(M / 128) * math.ceil(N / 128)
            # decode groups only: a 257-1024-token prefill chunk keeps the
            # prefill rule below (the target was measured on decode steps)
            if M <= 1024 and self.RESID_WG_TARGET and getattr(self, "decode", True):
                # decode groups above 256 rows: ~RESID_WG_TARGET 128x128 tiles,
                # at most one split per 1024 of K (at least 2).  512 rows, GEMM +
                # slab-folding norm (profiles/r2_resid512_splits.log): Llama-3 8B
                # down 119.7 -> 81.5 us, o-proj 44.2 -> 38.7; GPT-2 XL MLP-down
                # 54.7 -> 32.2 (the old rule gave 2 splits on the 128x64 ring)
                return max(1, min(math.ceil(self.RESID_WG_TARGET / tiles), max(2, K // 1024),
                                  K // 64 // 2 or 1))
            return max(1, min(math.ceil(256 / tiles), K // 64 // 2 or 1))
        if self.DEFER_RESID:
            # deferred slabs cost S x M x N x 4 B of writes + norm reads, so
            # fewer, longer splits win (measured, tools/microbench.py resid):
            # ~800 k per split, 4..8 splits
            return max(1, min(8, max(4, K // 800), K // 64))
        return self._sk_splits(M, N, K)

    def _sk_splits(self, M: int, N: int, K: int, nw: int = 1) -> int:
        nw = max(nw, 2 if M > self.NW2_ROWS else 1)  # mirrors sk_nw() in gemm.hip
        tiles = math.ceil(N / (64 * nw))  # >= SK_TARGET workgroups: never row-blocked
        target = self.SK_TARGET or max(128, 384 // max(1, self.concurrency))
        return max(1, min(math.ceil(target / tiles), K // 32 // self.SK_MIN_STEPS or 1))

    # non-residual decode GEMMs with a short K (GPT-2 small, K = 768) run tiled
    # at any row count above the GEMV: the split-K kernel's last-arriver
    # combine costs more than the k-loop it splits -- QKV 2304 x 768 at 8-128
    # rows 9.9-15.7 -> 7.6-8.0 us, MLP-up 3072 x 768 9.5-12.3 -> 7.8-8.3 us
    # (tools/bench_d256.py, profiles/r5_small_k_routing.log).  0 = off
    TILED_SHORT_K = int(os.environ.get("LSD_TILED_SHORT_K", "1024"))

    def _gemm_kw(self, M: int, N: int, K: int, nw: int = 1):
        bn = self._d256_bn(M, N, K)
        if bn:
            return self._d256_kind(bn), self._d256_splits(N, K, bn, self.D256_TARGET)
        if self._tiled(M, N) or (K <= self.TILED_SHORT_K and M <= self.SK_MAX_M and K % 64 == 0):
            return True, self._ring8_splits(M, N, K)
        return False, self._sk_splits(M, N, K, nw)

    def _ring8_splits(self, M: int, N: int, K: int) -> int:
        """K splits of a non-residual tiled decode GEMM on the 8-wave ring (1:
        unsplit; the host routing check is gemm.hip lsd_gemm_ring8_tiles)."""
        if not (self.RING8 == 2 and self.RING8_SK_TARGET and 128 < M <= self.SK_MAX_M and K % 64 == 0):
            return 1
        tiles = math.ceil(M / 128) * math.ceil(N / 64)
        S = max(1, min(round(self.RING8_SK_TARGET / tiles), K // 64 // 4, 4))
        if S > 1 and not self.C.gemm_ring8_tiles(M, N, K, S):
            return 1
        return S

    # ------------------------------------------------------------------
    def embed(self, ids, pos, wte, wpe):
        return self.C.embed(ids, pos, wte, wpe)

    def _norm(self, r: Residual, w, b, eps, rms: bool):
        if not r.pending and r.x.shape[0] <= self.GEMV_NORM_MAX_M and r.x.shape[1] % 8 == 0:
            return LazyNorm(r.x, w, b, eps, rms)
        self._flush_extra(r)
        slab, pb = (r.pending[0] if r.pending else (None, None))
        out = self.C.norm(r.x, slab, pb, w, b, eps, rms, None, True)
        r.pending.clear()
        return out

    def _flush_extra(self, r: Residual) -> None:
        while len(r.pending) > 1:
            slab, pb = r.pending.pop(0)
            self.C.norm(r.x, slab, pb, None, None, 0.0, True, None, False)

    def flush(self, r: Residual):
        for slab, pb in r.pending:
            self.C.norm(r.x, slab, pb, None, None, 0.0, True, None, False)
        r.pending.clear()
        return r.x

    def layernorm(self, r, w, b, eps):
        return self._norm(r, w, b, eps, False)

    def rmsnorm(self, r, w, eps):
        return self._norm(r, w, None, eps, True)

    def norm_rows(self, x, w, b, eps, rms: bool, rows=None):
        if rows is None and x.shape[0] <= self.GEMV_NORM_MAX_M and x.shape[1] % 8 == 0:
            return LazyNorm(x, w, b, eps, rms)
        return self.C.norm(x, None, None, w, b, eps, rms, rows, True)

    def materialize(self, xn):
        if isinstance(xn, LazyNorm):
            return self.C.norm(xn.x, None, None, xn.w, xn.b, xn.eps, xn.rms, None, True)
        return xn

    def _gemv_in(self, xn, K: int, epi: int):
        """(x, norm code, gamma, beta, eps) for a GEMV launch, or None when this
        GEMM does not run on the GEMV (the caller takes the MFMA path)."""
        M = xn.shape[0]
        if M > self.GEMV_MAX_M:
            return None
        if isinstance(xn, LazyNorm):
            if self.C.gemv_ok(M, K, epi, xn.code):
                return xn.x, xn.code, xn.w, xn.b, xn.eps
            xn = self.materialize(xn)
        if self.C.gemv_ok(M, K, epi, 0):
            return xn, 0, None, None, 0.0
        return None

    def qkv_kv_append(self, xn, w, b, cache_k, cache_v, meta, mcfg):
        g = self._gemv_in(xn, w.shape[1], EPI_QKV)
        if g is not None:
            x, nc, gw, gb, eps = g
            return self.C.gemv(x, w, b, EPI_QKV, nc, gw, gb, eps, None, cache_k, cache_v,
                               meta.token_slots, meta.token_pos, mcfg.q_size, mcfg.kv_size,
                               mcfg.head_dim, self._rope)
        xn = self.materialize(xn)
        if (self.BLASLT_QKV_MIN_M and getattr(self, "decode", False) and xn.shape[0] >= self.BLASLT_QKV_MIN_M
                and w.shape[1] >= self.BLASLT_QKV_MIN_K and xn.is_contiguous()):
            y = self.C.blaslt_f32(xn, w, self.lane)
            if y is not None:
                return self.C.qkv_post(y, b, cache_k, cache_v, meta.token_slots, meta.token_pos,
                                       mcfg.q_size, mcfg.kv_size, mcfg.head_dim, self._rope)
        tiled, splits = self._gemm_kw(xn.shape[0], w.shape[0], w.shape[1])
        return self.C.linear_qkv(xn, w, b, cache_k, cache_v, meta.token_slots, meta.token_pos,
                                 mcfg.q_size, mcfg.kv_size, mcfg.head_dim, self._rope,
                                 tiled, splits, self.counters)

    @classmethod
    def decode_attn_splits(cls, B: int, nh: int, n_kv: int, hd: int, max_ctx: int) -> int:
        """Context splits of a decode attention launch (a graph-captured
        property: max_ctx is the captured context bucket)."""
        G, items = nh // n_kv, B * n_kv
        if hd == 128 and G in (2, 4, 8):
            ms = 1
            if items < cls.ATTN_MFMA_SPLIT_BELOW:
                ms = max(1, min(math.ceil(cls.ATTN_MFMA_WAVES / items), math.ceil(max_ctx / 512), 256))
            if items * ms >= cls.ATTN_MFMA_MIN:
                return ms
        if items < cls.TARGET_BLOCKS:
            return min(math.ceil(cls.TARGET_BLOCKS / items), max(1, math.ceil(max_ctx / 256)))
        return 1

    def attention(self, q, cache_k, cache_v, meta):
        n_kv, hd = cache_k.shape[1], cache_k.shape[3]
        nh = q.shape[1] // hd
        if meta.is_decode:
            splits = self.decode_attn_splits(meta.num_seqs, nh, n_kv, hd, meta.max_ctx)
            return self.C.attn_decode(q, cache_k, cache_v, meta.seq_slots, meta.token_pos, nh, splits)
        tiles = getattr(meta, "_tiles", None)
        if tiles is None:
            tiles = prefill_tiles(meta).to(q.device)
            meta._tiles = tiles
        return self.C.attn_prefill(q, cache_k, cache_v, tiles, meta.seq_slots, meta.q_start,
                                   meta.cu_q, nh)

    # Decode attention fused with the output projection + residual add at
    # <= ATTN_OPROJ_MAX_M rows (attention.hip attn_oproj_kernel): one launch
    # instead of attention + out-projection GEMV.  Off by default: the
    # cross-block hand-off of the per-head partials (write-through stores,
    # ticket, last-arriver reload) costs more than the kernel boundary it
    # removes -- single stream GPT-2 XL 1.385 -> 1.570 ms, small 0.290 ->
    # 0.316, Llama-3 8B 3.19 -> 3.37 (profiles/r3_attn_oproj_single_stream.log)
    ATTN_OPROJ_MAX_M = int(os.environ.get("LSD_ATTN_OPROJ_MAX_M", "0"))

    def attention_oproj(self, q, cache_k, cache_v, meta, w, b, r: Residual) -> bool:
        """x += attention(q) @ w^T + b in one kernel; False = not applicable
        (the caller runs attention + linear_residual)."""
        M = q.shape[0]
        if not meta.is_decode or M > min(self.ATTN_OPROJ_MAX_M, 4) or M < 1:
            return False
        n_kv, hd = cache_k.shape[1], cache_k.shape[3]
        nh = q.shape[1] // hd
        G = nh // n_kv
        if not ((hd == 64 and G == 1) or (hd == 128 and G in (1, 2, 4, 8))):
            return False
        if r.pending:
            self.flush(r)
        N = w.shape[0]
        C = max(1, -(-256 // n_kv))           # ~256 blocks: n_kv heads x C column chunks
        nc = -(-(-(-N // C)) // 16) * 16      # chunk columns, a multiple of 16
        self.C.attn_oproj(q, cache_k, cache_v, meta.seq_slots, meta.token_pos, nh, w, b, r.x, nc,
                          self.counters)
        return True

    def linear(self, a, w, b=None, act: str = "none"):
        code = _EPI[act]
        g = self._gemv_in(a, w.shape[1], code)
        if g is not None:
            x, nc, gw, gb, eps = g
            return self.C.gemv(x, w, b, code, nc, gw, gb, eps, None, None, None, None, None,
                               0, 0, 0, None)
        a = self.materialize(a)
        dec_gelu = (code == 1 and self.BLASLT_DECODE_GELU_MIN_M and getattr(self, "decode", False)
                    and a.shape[0] >= self.BLASLT_DECODE_GELU_MIN_M)
        if ((code == 1 and self._blaslt(a.shape[0]) and a.shape[0] >= self.BLASLT_GELU_MIN_M) or dec_gelu) \
                and a.is_contiguous():
            y = self.C.blaslt_linear(a, w, b, code, self.lane)
            if y is not None:
                return y
        if code == 2 and self.BLASLT_SILU_MIN_M and self.BLASLT_SILU_MIN_M <= a.shape[0] <= self.BLASLT_SILU_MAX_M \
                and getattr(self, "decode", False) and a.is_contiguous() and w.shape[0] % 32 == 0:
            y = self.C.blaslt_linear(a, w, b, 0, self.lane)
            if y is not None:
                return self.C.silu_mul(y)
        tiled, splits = self._gemm_kw(a.shape[0], w.shape[0], w.shape[1], 2 if code == 2 else 1)
        return self.C.linear(a, w, b, code, tiled, splits, self.counters)

    def _blaslt(self, M: int) -> bool:
        return bool(self.BLASLT_MIN_M) and M >= self.BLASLT_MIN_M and not getattr(self, "decode", True)

    def linear_residual(self, a, w, b, r: Residual) -> None:
        M, K = a.shape
        N = w.shape[0]
        if self._gemv_in(a, K, EPI_RESID) is not None:  # adds straight into r.x
            self.C.gemv(a, w, b, EPI_RESID, 0, None, None, 0.0, r.x, None, None, None, None,
                        0, 0, 0, None)
            return
        if self._blaslt(M) and K >= self.BLASLT_RESID_MIN_K and a.is_contiguous() \
                and self.C.blaslt_residual(a, w, b, r.x, self.lane):
            return
        splits = self._resid_splits(M, N, K)
        tiled = self._tiled(M, N)
        bn = self._d256_bn(M, N, K) if self.D256_RESID else 0
        if bn:
            tiled = self._d256_kind(bn)
        # decode split-K: hand the S partial slabs to the next norm (which
        # reads the rows anyway) instead of a last-arriver reduce in the GEMM
        defer = self.DEFER_RESID and not tiled and splits > 1
        if self.PREFILL_SLAB and tiled and splits == 1 and not getattr(self, "decode", True) and M > 256:
            # prefill: the GEMM writes one bf16 slab (the norm that follows folds
            # it into the fp32 stream) instead of an fp32 read-modify-write of
            # the residual in its epilogue
            defer = True
        slab = self.C.linear_residual(a, w, b, r.x, splits, tiled, self.counters, defer)
        if slab is not None:
            r.pending.append((slab, b))

    def logits(self, xn, w):
        g = self._gemv_in(xn, w.shape[1], EPI_F32)
        if g is not None:
            x, nc, gw, gb, eps = g
            return self.C.gemv(x, w, None, EPI_F32, nc, gw, gb, eps, None, None, None, None,
                               None, 0, 0, 0, None)
        xn = self.materialize(xn)
        # vocab-wide N: the 128x128 LDS-tiled kernel fills the chip without
        # split-K and reads the activation rows once per 128 columns instead
        # of once per 64 -- measured 41.8 vs 64.2 us at M = 128 (GPT-2 XL),
        # 222.7 vs 300.3 us for Llama-3 8B (tools/microbench.py lmhead)
        if w.shape[0] >= 16384 and w.shape[1] % 64 == 0:
            tiled, splits = True, 1
        else:
            tiled, splits = self._gemm_kw(xn.shape[0], w.shape[0], w.shape[1])
        if not (self.SEGMAX and tiled and w.shape[0] % 8 == 0):
            return self.C.linear_f32(xn, w, tiled, splits, self.counters)
        # the epilogue also writes each 8-logit segment's maximum; the sampler
        # derives its top-k threshold from them and reads only the segments
        # that reach it (attached to the logits: a slice drops it, and the
        # sampler then scans the full rows)
        seg = torch.empty(xn.shape[0], w.shape[0] // 8, dtype=torch.float32, device=xn.device)
        out = self.C.linear_f32(xn, w, tiled, splits, self.counters, seg)
        out._lsd_segmax = seg
        return out

    def sample(self, logits, samp, vocab: int):
        return self.C.sample(logits, vocab, samp.temperature, samp.top_k, samp.greedy,
                             samp.seeds, samp.step, getattr(logits, "_lsd_segmax", None))

    def sample_into(self, logits, samp, vocab: int, out, meta=None) -> None:
        # one kernel: draw into `out`, advance the per-row sampler counters
        # and (meta given) the decode batch's positions
        self.C.sample_into(logits, vocab, samp.temperature, samp.top_k, samp.greedy,
                           samp.seeds, samp.step, out, getattr(samp, "active", None),
                           meta.token_pos if meta is not None else None,
                           getattr(logits, "_lsd_segmax", None))

    def gather_rows(self, x, idx):
        return x.index_select(0, idx.long())
