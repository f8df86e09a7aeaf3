"""Per-device engine: owns one libmmf_hip handle (weights, workspaces, Truth-Vault) and exposes
the five signals as batched tensor calls on torch device tensors (torch = device memory and
streams only; all arithmetic runs in the HIP kernels of libmmf_hip.so)."""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import numpy as np
import torch

from . import hip, io_utils
from .hip import check, ptr, stream_ptr

SCORE_KEYS = ("ai_score", "misinfo_score", "deepfake_score", "clip_similarity", "vault_discrepancy")


def _as_np(v) -> np.ndarray:
    if isinstance(v, torch.Tensor):
        v = v.detach().cpu()
        return v.numpy() if v.dtype == torch.int64 else v.float().numpy()
    return np.asarray(v)


class Engine:
    """MI355X replica of the MisinfoForensics models on one device."""

    EFFNET_PRECISIONS = ("auto", "fp16", "fp32")
    # RoBERTa stream / operand precision -> option text_hilo (capi.cpp run_text / run_text_precise):
    # "auto" = the LayerNorm-bound layout (-1: fp16 or split stream) unless the load-time calibration
    # selects "precise"; the others pin the mode ("fp16" / "split" also skip packing the precise weights)
    TEXT_PRECISIONS = {"auto": -1, "fp16": 0, "split": 1, "precise": 2}

    def __init__(self, device: int = 0, detector_state=None, clip_state=None, eos_token_id: int = 49407,
                 max_batch: int = 256, max_text_len: int = 128, max_clip_len: int = 77,
                 effnet_precision: str = "auto", text_precision: str = "auto"):
        if effnet_precision not in self.EFFNET_PRECISIONS:
            raise ValueError(f"effnet_precision must be one of {self.EFFNET_PRECISIONS}, got {effnet_precision!r}")
        if text_precision not in self.TEXT_PRECISIONS:
            raise ValueError(f"text_precision must be one of {tuple(self.TEXT_PRECISIONS)}, got {text_precision!r}")
        self.lib = hip.load()
        self.device = torch.device("cuda", device)
        torch.cuda.set_device(self.device)
        h = ctypes.c_void_p()
        check(self.lib.mmf_create(device, ctypes.byref(h)), "mmf_create")
        self.h = h
        self.eos_token_id = eos_token_id
        self.effnet_precision = effnet_precision
        self.text_precision = text_precision
        self.effnet_check = None
        self.text_check = None
        # an MMF_TEXT_HILO / MMF_EFFNET_FP32 environment value pins the tower under "auto"
        # (no calibration overrides it); so does a set_option of text_hilo / effnet_fp32 made after
        # the engine's own last write (_auto_set records those writes)
        self._auto_set = {}
        if text_precision == "auto" and os.environ.get("MMF_TEXT_HILO"):
            self.text_precision = "pinned"
        else:
            self._auto_write("text_hilo", self.TEXT_PRECISIONS[text_precision])
        if effnet_precision == "auto" and os.environ.get("MMF_EFFNET_FP32"):
            self.effnet_precision = "pinned"
        elif effnet_precision == "auto":
            self._auto_set["effnet_fp32"] = self.get_option("effnet_fp32")
        self.clip_stream_check = None
        self.vault_n = 0
        if detector_state is not None:
            self.load_state(detector_state, "")
        if clip_state is not None:
            self.load_state(clip_state, "clip.")
        self.finalize()
        self.reserve(max_batch, max_text_len, max_clip_len)
        if clip_state is not None:
            self.check_clip_streams()
        self.calibrate(("text", "effnet") if detector_state is not None else ())

    # ------------------------------------------------------------------ weights
    def load_state(self, state: Dict, prefix: str = "") -> None:
        for name, v in state.items():
            a = _as_np(v)
            if a.dtype == np.int64:
                dt = 1
            else:
                a = np.ascontiguousarray(a, dtype=np.float32)
                dt = 0
            shape = (ctypes.c_int64 * max(1, a.ndim))(*a.shape)
            check(self.lib.mmf_load_tensor(self.h, (prefix + name).encode(), dt, a.ndim, shape,
                                           a.ctypes.data_as(ctypes.c_void_p)), f"load {prefix + name}")

    def finalize(self) -> None:
        check(self.lib.mmf_finalize(self.h, int(self.eos_token_id)), "mmf_finalize")

    @property
    def ready(self) -> int:
        return self.lib.mmf_ready(self.h)

    # fp16 CLIP streams: largest tolerated change of an image-text cosine (the quantity clip_similarity
    # and the vault scores are made of) between fp16 and fp32 residual streams -- half of the
    # north-star 1e-3 (the ordinary synthetic draw measures 2.3e-4, an outlier-feature draw 1.3e-4)
    CLIP_STREAM_TOL = 5e-4

    def check_clip_streams(self, n: int = 8) -> dict:
        """Load-time guard of the fp16 CLIP residual streams (option clip_res16).

        The pre-LN stream is a running sum, so unlike RoBERTa's post-LN stream no LayerNorm
        parameter bounds it: trained weights with outlier features can push it past fp16's range
        (65504) or far enough up that its rounding matters.  A calibration forward measures it: both
        CLIP towers on n seeded images / captions with fp16 streams and again with fp32 streams; if
        an embedding is non-finite or any of the n x n image-text cosines moves by more than
        CLIP_STREAM_TOL, the fp32 streams stay selected.  Returns (and keeps as `clip_stream_check`)
        the measured change."""
        from . import synthetic as syn
        if self.get_option("clip_res16") != 1:
            return self.clip_stream_check or {}
        n = max(1, min(n, self.max_batch))
        imgs = torch.from_numpy(syn.images(n, 4099)).to(self.device)
        ids, mask = syn.clip_ids(n, min(77, self.max_clip_len), 4099)

        def cosines():
            e = self.clip_image(imgs).double()
            t = self.clip_text(ids, mask).double()
            return e, t, e @ t.T  # unit rows: cosines
        e16, t16, c16 = cosines()
        self.set_option("clip_res16", 0)
        e32, t32, c32 = cosines()
        finite = bool(torch.isfinite(e16).all() and torch.isfinite(t16).all())
        dcos = float((c16 - c32).abs().max()) if finite else float("inf")
        demb = float(max((e16 - e32).abs().max(), (t16 - t32).abs().max())) if finite else float("inf")
        ok = finite and dcos <= self.CLIP_STREAM_TOL
        if ok:
            self.set_option("clip_res16", 1)
        self.clip_stream_check = {"max_dcos": dcos, "max_demb": demb, "fp16_streams": ok, "rows": n}
        return self.clip_stream_check

    def clip_stream_overflow(self, *outputs) -> bool:
        """Run-time overflow trap of the fp16 CLIP streams: the load-time calibration
        measures 8 seeded inputs, so it bounds nothing for later ones.  An input that drives a
        stream past fp16's range turns the embedding non-finite, and clip_similarity / the vault
        scores with it.  The synchronous API paths (which read their results back anyway) pass
        their CLIP outputs here: if fp16 streams are selected and any value is non-finite, the
        engine switches to fp32 streams for good and returns True, and the caller re-runs the
        batch.  Drift short of overflow is what the calibration alone covers.  An output
        may be a device tensor or a host array the caller already read back (checked on the host:
        no device launch or extra synchronisation)."""
        if self.get_option("clip_res16") != 1:
            return False

        def finite(v) -> bool:
            return bool(np.isfinite(v).all()) if isinstance(v, np.ndarray) else bool(torch.isfinite(v).all())
        if all(finite(v) for v in outputs if v is not None):
            return False
        self.set_option("clip_res16", 0)
        self.clip_stream_check = dict(self.clip_stream_check or {}, fp16_streams=False, runtime_overflow=True)
        return True

    # fp16 EfficientNet tower: largest tolerated change of deepfake_score against the fp32 tower on
    # the calibration images (half the north-star bar; the ordinary draw measures ~1e-4 over 256)
    EFFNET_TOL = 5e-4

    def _auto_write(self, name: str, value: int) -> None:
        self.set_option(name, value)
        self._auto_set[name] = int(value)

    def _pinned(self, name: str) -> bool:
        """True when the option was changed since the engine last wrote it (a user pin)."""
        return name in self._auto_set and self.get_option(name) != self._auto_set[name]

    def calibrate(self, components=("effnet",)) -> None:
        """Load-time precision selection for re-packed components (called at construction and by
        the detector's sync after every re-pack: trained weights reach the engine through
        misinfo_forensics.py:175-186 / 285-303 after construction)."""
        if "text" in components and self.ready & 1:
            self.check_text_precision()
        if "effnet" in components and self.ready & 2:
            self.check_effnet_precision()

    # RoBERTa: largest tolerated change of ai_score / misinfo_score between the fast layout and the
    # precise mode on the calibration texts (half the north-star bar)
    TEXT_TOL = 5e-4

    # precise-mode GEMM kinds (option text_prec_mask: bit k = kind k on hi / lo activations, bit k + 4 =
    # also on W_lo; kinds QKV, out-proj, FFN-1, FFN-2) and their relative GEMM cost (the K loop is 1x /
    # 2x / 3x): the calibration keeps the cheapest mask within TEXT_TOL of the full mode (255)
    PREC_KIND_COST = (3, 1, 4, 4)
    PREC_FULL = 255

    @classmethod
    def _mask_cost(cls, m: int) -> int:
        return sum(c * (1 + (m >> k & 1) + (m >> k & 1) * (m >> (k + 4) & 1)) for k, c in enumerate(cls.PREC_KIND_COST))

    @classmethod
    def _prec_masks(cls):
        """Every operand mask below the full mode, cheapest first (3 levels per kind)."""
        import itertools
        ms = [sum((lv >= 1) << k | (lv == 2) << (k + 4) for k, lv in enumerate(lvls))
              for lvls in itertools.product((0, 1, 2), repeat=4)]
        return sorted((m for m in ms if m != cls.PREC_FULL), key=lambda m: (cls._mask_cost(m), m))

    def check_text_precision(self, n: int = 64) -> dict:
        """Load-time selection of the RoBERTa text mode.  The
        fp16-operand design holds 1e-3 only while the LayerNorms do not amplify operand rounding: a
        checkpoint with one channel dominating every LayerNorm (gamma ~7: DESIGN.md §4) moves the
        scores by 1.6e-3 even on the split stream.  With text_precision "auto", on n seeded texts of
        128 tokens:
          1. the fast layout (fp16 or split stream, from the LayerNorm bound) against the full
             precise mode (fp32 stream / LayerNorm / attention, every GEMM on ~22-bit hi / lo
             operands); within TEXT_TOL on every score -> the fast layout, and the precise weights
             are released (the run-time trap falls back to the precise mode on fp16 operands,
             which needs none of them);
          2. otherwise every cheaper operand mask (option text_prec_mask: which GEMM kinds read hi / lo
             operands, the rest fp16) against the full mode; the cheapest within TEXT_TOL is
             selected and only its kinds' weights stay packed.
        A user pin (text_precision other than "auto", MMF_TEXT_HILO, or a set_option of text_hilo
        after the engine's last write) is left alone."""
        from . import synthetic as syn
        if self.text_precision != "auto" or self._pinned("text_hilo"):
            self.text_check = {"mode": self.text_precision if self.text_precision != "auto" else "pinned",
                               "calibrated": False}
            return self.text_check
        self._auto_write("text_hilo", -1)
        n = max(1, n)
        L = min(128, self.max_text_len)
        ids, mask = syn.roberta_ids(n, L, 6007, [L, L // 2, 17, 5])

        def scores():
            return torch.cat([self.text_forward(ids[i:i + self.max_batch], mask[i:i + self.max_batch])[2].double()
                              for i in range(0, n, self.max_batch)])

        def dist(a, b):
            return float((a - b).abs().max()) if bool(torch.isfinite(a).all()) else float("inf")
        names = {0: "fp16", 1: "split", 2: "precise"}
        fast = scores()
        fast_mode = self.get_option("text_hilo_effective")
        packed = self.get_option("text_precise_packed")
        if packed != 15:  # (weights packed under a pinned layout: nothing to compare against)
            self.text_check = {"mode": names[fast_mode], "calibrated": False, "precise_packed": packed}
            return self.text_check
        self.set_option("text_prec_mask", self.PREC_FULL)
        self._auto_write("text_hilo", 2)
        full = scores()
        d = dist(fast, full)
        self.text_check = {"max_dscore": d, "fast_layout": names[fast_mode], "texts": n, "calibrated": True}
        if d <= self.TEXT_TOL:
            self._auto_write("text_hilo", -1)
            self.set_option("text_precise_packed", 0)  # the +510 MB go when the mode is not used
            self.text_check["mode"] = names[fast_mode]
            return self.text_check
        tried = {}
        best = self.PREC_FULL
        for m in self._prec_masks():
            self.set_option("text_prec_mask", m)
            tried[m] = dist(scores(), full)
            if tried[m] <= self.TEXT_TOL:
                best = m
                break
        self.set_option("text_prec_mask", best)
        self.set_option("text_precise_packed", best & 15)
        self.text_check.update(mode="precise", prec_mask=best, mask_dscore=tried,
                               cost_vs_full=self._mask_cost(best) / self._mask_cost(self.PREC_FULL))
        return self.text_check

    def text_overflow(self, scores) -> bool:
        """Run-time overflow trap of the fast RoBERTa layouts (the counterpart of
        clip_stream_overflow).  The load-time calibration bounds the drift on its seeded texts; an
        input whose branch output passes fp16's range (a token driving an FFN-2 row past 65504) turns
        that text's scores non-finite.  Given text scores the caller already read back: if a fast
        layout is selected and any is non-finite, the engine switches to the precise mode for good
        (fp32 stream and branch outputs; hi / lo operands for the kinds still packed, fp16 for the
        rest) and returns True, and the caller re-runs the batch.  A pinned layout is left alone."""
        if self.get_option("text_hilo_effective") >= 2 or self._pinned("text_hilo"):
            return False
        if bool(np.isfinite(np.asarray(scores)).all()):
            return False
        packed = self.get_option("text_precise_packed")
        self.set_option("text_prec_mask", packed | packed << 4)
        self._auto_write("text_hilo", 2)
        self.text_check = dict(self.text_check or {}, mode="precise", runtime_overflow=True,
                               prec_mask=self.get_option("text_prec_mask"))
        return True

    def effnet_overflow(self, scores) -> bool:
        """Run-time overflow trap of the fp16 EfficientNet tower: given
        deepfake scores the caller already read back, a non-finite one under the fp16 tower switches
        the engine to the fp32 tower for good and returns True (the caller re-runs the batch).  An
        image whose activation passes fp16's range (a saturated colour on a high-gain stem channel)
        is what the load-time calibration on seeded images cannot see.  A pinned tower is left
        alone."""
        if self.get_option("effnet_fp32") != 0 or self.effnet_precision != "auto" or self._pinned("effnet_fp32"):
            return False
        if bool(np.isfinite(np.asarray(scores)).all()):
            return False
        self._auto_write("effnet_fp32", 1)
        self.effnet_check = dict(self.effnet_check or {}, tower="fp32", runtime_overflow=True)
        return True

    def scores_overflow(self, scores5) -> bool:
        """All three run-time traps on an analyze_batch result read back to the host ([B, 5]: ai,
        misinfo, deepfake, clip_similarity, vault): True when any tower switched precision (the
        caller re-runs the batch once)."""
        s = np.asarray(scores5)
        hit = self.text_overflow(s[:, :2])
        hit = self.effnet_overflow(s[:, 2]) or hit
        return self.clip_stream_overflow(s[:, 3]) or hit

    def check_effnet_precision(self, n: int = 64) -> dict:
        """Load-time guard of the fp16 EfficientNet tower (the counterpart of
        check_clip_streams).  A BN-conditioned tower is insensitive to fp16 activation storage; a
        chaotic one (logits of O(100): He-gain draws) amplifies it to O(0.1).  With
        effnet_precision "auto" both towers run on n seeded calibration images; if any deepfake_score
        is non-finite or moves by more than EFFNET_TOL, the fp32 tower stays selected.  "fp16" /
        "fp32" pin the tower without measuring.  Returns (and keeps as `effnet_check`) the result."""
        from . import synthetic as syn
        if self.effnet_precision != "auto" or self._pinned("effnet_fp32"):
            if self.effnet_precision in ("fp16", "fp32"):
                self.set_option("effnet_fp32", int(self.effnet_precision == "fp32"))
            self.effnet_check = {"tower": self.effnet_precision if self.effnet_precision != "auto" else "pinned",
                                 "calibrated": False}
            return self.effnet_check
        n = max(1, n)
        imgs = torch.from_numpy(syn.images(n, 5003)).to(self.device)

        def scores(fp32: int):
            self._auto_write("effnet_fp32", fp32)
            out = []
            for i in range(0, n, self.max_batch):
                out.append(self.effnet_forward(imgs[i:i + self.max_batch])[1].double())
            return torch.cat(out)
        s16, s32 = scores(0), scores(1)
        finite = bool(torch.isfinite(s16).all())
        d = float((s16 - s32).abs().max()) if finite else float("inf")
        ok = finite and d <= self.EFFNET_TOL
        self._auto_write("effnet_fp32", 0 if ok else 1)
        self.effnet_check = {"max_ddeepfake": d, "tower": "fp16" if ok else "fp32", "images": n, "calibrated": True}
        return self.effnet_check

    # ------------------------------------------------------------------ options / accounting
    def set_option(self, name: str, value: int) -> None:
        """A/B switches of the library (include/mmf_hip.h: mmf_set_option)."""
        check(self.lib.mmf_set_option(self.h, name.encode(), int(value)), f"mmf_set_option({name})")

    def get_option(self, name: str) -> int:
        v = ctypes.c_int()
        check(self.lib.mmf_get_option(self.h, name.encode(), ctypes.byref(v)), f"mmf_get_option({name})")
        return v.value

    @property
    def device_bytes(self) -> int:
        """Device memory owned by this handle (weights, workspaces, vault)."""
        return int(self.lib.mmf_device_bytes(self.h))

    def reserve(self, max_batch: int, max_text_len: int = 128, max_clip_len: int = 77) -> None:
        check(self.lib.mmf_reserve(self.h, max_batch, max_text_len, max_clip_len), "mmf_reserve")
        self.max_batch, self.max_text_len, self.max_clip_len = max_batch, max_text_len, max_clip_len

    # ------------------------------------------------------------------ vault
    def set_vault(self, embeddings: np.ndarray, title_ids=None, title_mask=None) -> None:
        """Rows normalised once, exactly as the reference does on every search call (numpy, in the
        vault's own dtype: io_utils.vault_unit_rows), then uploaded as float32."""
        v = np.ascontiguousarray(io_utils.vault_unit_rows(_as_np(embeddings)), dtype=np.float32)
        check(self.lib.mmf_set_vault_normalized(self.h, v.ctypes.data_as(ctypes.c_void_p), v.shape[0], v.shape[1]),
              "mmf_set_vault_normalized")
        self.vault_n = v.shape[0]
        if title_ids is not None:
            ids = self._i32(title_ids)
            mask = self._i32(title_mask)
            check(self.lib.mmf_set_vault_titles(self.h, ptr(ids), ptr(mask), ids.shape[0], ids.shape[1],
                                                stream_ptr()), "mmf_set_vault_titles")

    # ------------------------------------------------------------------ host-input geometry
    def resize_supported(self, width: int, height: int) -> bool:
        """Whether mmf_resize_pil's tap budget covers a width x height image (both geometries)."""
        return bool(self.lib.mmf_resize_supported(int(width), int(height)))

    def resize_images(self, images, effnet: bool = True, clip: bool = True):
        """Decoded uint8 images (HxWx3 RGB or HxWx4 RGBX numpy arrays -- all of one kind --, any
        sizes) -> device uint8 [B,224,224,3] EfficientNet squash-resize and CLIP shortest-edge +
        centre-crop windows, bit-exact with Pillow (mmf_resize_pil).  The images cross PCIe once,
        packed (threaded copies) into a pinned staging buffer."""
        arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
        ps = arrs[0].shape[2] if arrs else 3
        for a in arrs:
            if not (a.ndim == 3 and a.shape[2] == ps and ps in (3, 4)):
                raise ValueError(f"expected HxWx{ps} uint8, got {a.shape}")
        sizes = [a.nbytes for a in arrs]
        offs = np.zeros(len(arrs), np.int64)
        if arrs:
            offs[1:] = np.cumsum(sizes)[:-1]
        total = int(sum(sizes)) or 1
        if getattr(self, "_rs_host", None) is None or self._rs_host.numel() < total:
            self._rs_host = torch.empty(total, dtype=torch.uint8).pin_memory()
        host = self._rs_host.numpy()

        def pack(i):
            np.copyto(host[offs[i]:offs[i] + sizes[i]], arrs[i].reshape(-1))
        if total > (8 << 20) and len(arrs) > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=min(16, len(arrs))) as ex:
                list(ex.map(pack, range(len(arrs))))
        else:
            for i in range(len(arrs)):
                pack(i)
        src = self._rs_host[:total].to(self.device, non_blocking=True)
        wh = np.array([[a.shape[1], a.shape[0]] for a in arrs], np.int32).reshape(-1)
        B = len(arrs)
        eff = torch.empty((B, 224, 224, 3), dtype=torch.uint8, device=self.device) if effnet else None
        clp = torch.empty((B, 224, 224, 3), dtype=torch.uint8, device=self.device) if clip else None
        check(self.lib.mmf_resize_pil(self.h, ptr(src), offs.ctypes.data_as(ctypes.c_void_p),
                                      wh.ctypes.data_as(ctypes.c_void_p), B, ps, ptr(eff), ptr(clp), stream_ptr()),
              "mmf_resize_pil")
        return eff, clp

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _tensor(x) -> torch.Tensor:
        # a read-only numpy view (an Arrow / PIL export, np.broadcast_to) is copied rather than
        # wrapped: torch cannot wrap non-writable memory without a UserWarning per process
        if isinstance(x, np.ndarray) and not x.flags.writeable:
            x = x.copy()
        return torch.as_tensor(x)

    def _i32(self, x) -> torch.Tensor:
        return self._tensor(x).to(self.device, torch.int32).contiguous()

    def _u8(self, x) -> torch.Tensor:
        t = self._tensor(x)
        if not (t.dtype == torch.uint8 and t.dim() == 4 and tuple(t.shape[1:]) == (224, 224, 3)):
            raise ValueError(f"images must be uint8 [B,224,224,3], got {tuple(t.shape)} {t.dtype}")
        return t.to(self.device).contiguous()

    def _f32(self, *shape) -> torch.Tensor:
        return torch.empty(shape, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ signals
    def text_forward(self, ids, mask):
        ids, mask = self._i32(ids), self._i32(mask)
        B, L = ids.shape
        ai, mi, sc = self._f32(B, 2), self._f32(B, 2), self._f32(B, 2)
        check(self.lib.mmf_text_forward(self.h, ptr(ids), ptr(mask), B, L, ptr(ai), ptr(mi), ptr(sc),
                                        stream_ptr()), "mmf_text_forward")
        return ai, mi, sc

    def effnet_forward(self, img):
        img = self._u8(img)
        B = img.shape[0]
        lg, sc = self._f32(B, 2), self._f32(B)
        check(self.lib.mmf_effnet_forward(self.h, ptr(img), B, ptr(lg), ptr(sc), stream_ptr()), "mmf_effnet_forward")
        return lg, sc

    def effnet_forward_f32(self, x):
        """Normalised fp32 NCHW input (detector.forward_image semantics)."""
        x = torch.as_tensor(x, dtype=torch.float32).to(self.device).contiguous()
        if not (x.dim() == 4 and tuple(x.shape[1:]) == (3, 224, 224)):
            raise ValueError(f"expected [B,3,224,224], got {tuple(x.shape)}")
        B = x.shape[0]
        lg, sc = self._f32(B, 2), self._f32(B)
        check(self.lib.mmf_effnet_forward_f32(self.h, ptr(x), B, ptr(lg), ptr(sc), stream_ptr()),
              "mmf_effnet_forward_f32")
        return lg, sc

    def clip_image(self, img):
        img = self._u8(img)
        e = self._f32(img.shape[0], 512)
        check(self.lib.mmf_clip_image(self.h, ptr(img), img.shape[0], ptr(e), stream_ptr()), "mmf_clip_image")
        return e

    def clip_text(self, ids, mask):
        ids, mask = self._i32(ids), self._i32(mask)
        e = self._f32(ids.shape[0], 512)
        check(self.lib.mmf_clip_text(self.h, ptr(ids), ptr(mask), ids.shape[0], ids.shape[1], ptr(e),
                                     stream_ptr()), "mmf_clip_text")
        return e

    def clip_consistency(self, img, ids, mask, out: Optional[dict] = None) -> dict:
        """analyze_consistency over a batch: {img_emb, txt_emb [B,512] unit, sim [B]} (one call,
        the CLIP text tower on a concurrent stream)."""
        img = self._u8(img)
        ids, mask = self._i32(ids), self._i32(mask)
        B = img.shape[0]
        if out is None:
            out = {"img_emb": self._f32(B, 512), "txt_emb": self._f32(B, 512), "sim": self._f32(B)}
        check(self.lib.mmf_clip_consistency(self.h, ptr(img), ptr(ids), ptr(mask), B, ids.shape[1],
                                            ptr(out["img_emb"]), ptr(out["txt_emb"]), ptr(out["sim"]), stream_ptr()),
              "mmf_clip_consistency")
        return out

    def vault_topk(self, q_unit: torch.Tensor, k: int = 5, thresh: float = 0.85, text_emb=None):
        q = q_unit.contiguous()
        B = q.shape[0]
        sims, idx = self._f32(B, k), torch.empty((B, k), dtype=torch.int32, device=self.device)
        disc, tsim = self._f32(B), self._f32(B)
        check(self.lib.mmf_vault_topk(self.h, ptr(q), B, k, float(thresh), ptr(sims), ptr(idx), ptr(disc),
                                      ptr(text_emb), ptr(tsim), stream_ptr()), "mmf_vault_topk")
        return sims, idx, disc, tsim

    def fusion(self, x5):
        x5 = torch.as_tensor(x5, dtype=torch.float32).to(self.device).contiguous()
        B = x5.shape[0]
        probs, conf = self._f32(B, 2), self._f32(B)
        verdict = torch.empty(B, dtype=torch.int32, device=self.device)
        rule = torch.empty(B, dtype=torch.int32, device=self.device)
        check(self.lib.mmf_fusion(self.h, ptr(x5), B, ptr(probs), ptr(verdict), ptr(conf), ptr(rule), stream_ptr()),
              "mmf_fusion")
        return probs, verdict, conf, rule

    def analyze_batch(self, rob_ids, rob_mask, clip_ids, clip_mask, img, img_clip=None,
                      out: Optional[dict] = None) -> dict:
        """Text+image pairs through all five signals + fusion (misinfo_forensics.py:767-927)."""
        rob_ids, rob_mask = self._i32(rob_ids), self._i32(rob_mask)
        clip_ids, clip_mask = self._i32(clip_ids), self._i32(clip_mask)
        img = self._u8(img)
        img_clip = self._u8(img_clip) if img_clip is not None else None
        B = rob_ids.shape[0]
        if out is None:
            out = self.alloc_outputs(B)
        check(self.lib.mmf_analyze_batch(
            self.h, ptr(rob_ids), ptr(rob_mask), rob_ids.shape[1], ptr(clip_ids), ptr(clip_mask), clip_ids.shape[1],
            ptr(img), ptr(img_clip), B, ptr(out["scores"]), ptr(out["text_similarity"]), ptr(out["probs"]),
            ptr(out["verdict"]), ptr(out["confidence"]), ptr(out["rule"]), ptr(out["top_sims"]),
            ptr(out["top_idx"]), stream_ptr()), "mmf_analyze_batch")
        return out

    def alloc_outputs(self, B: int) -> dict:
        d = self.device
        return {"scores": self._f32(B, 5), "text_similarity": self._f32(B), "probs": self._f32(B, 2),
                "verdict": torch.empty(B, dtype=torch.int32, device=d), "confidence": self._f32(B),
                "rule": torch.empty(B, dtype=torch.int32, device=d), "top_sims": self._f32(B, 5),
                "top_idx": torch.empty((B, 5), dtype=torch.int32, device=d)}

    def host_pipeline(self, B: int, Lr: int, Lc: int = 77) -> "HostPipeline":
        return HostPipeline(self, B, Lr, Lc)

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.mmf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class HostPipeline:
    """analyze_batch over batches that start in HOST memory (the boundary of analyze_pairs and of a
    serving loop): three device input slots (MMF_PIPE_SLOTS), H2D copies of batch i+1 on a copy stream while batch i
    computes on the current stream (ids int32 + uint8 images, ~38.6 MB per 256 pairs), results
    copied back into pinned host tensors.  Host inputs should be pinned (`torch.Tensor.pin_memory`)
    for the copies to run asynchronously."""

    _IN = ("rid", "rm", "cid", "cm", "img")

    def __init__(self, eng: Engine, B: int, Lr: int, Lc: int = 77, d2h_stream: Optional[bool] = None):
        self.eng, self.B = eng, B
        # result copies on a stream of their own (behind the batch's compute, beside the next batch's)
        # instead of in the compute stream; MMF_D2H_STREAM=0 restores the in-stream copies (A/B)
        if d2h_stream is None:
            d2h_stream = os.environ.get("MMF_D2H_STREAM", "1") != "0"
        self.d2h = torch.cuda.Stream(device=eng.device) if d2h_stream else None
        d = eng.device
        shapes = {"rid": ((B, Lr), torch.int32), "rm": ((B, Lr), torch.int32), "cid": ((B, Lc), torch.int32),
                  "cm": ((B, Lc), torch.int32), "img": ((B, 224, 224, 3), torch.uint8)}
        # input/output slots = batches in flight (MMF_PIPE_SLOTS, default 3): the copy of batch i+1 beside
        # the compute of batch i, and the host one more batch ahead.  With 2, a host hiccup longer than
        # one batch's compute left the device idle: bench headline 18,365 -> 18,562 pairs/s (3
        # interleaved processes), now level with the HBM-resident rate (profiles/r04_ab_pipe_slots.txt, git history at 168304c)
        self.n = max(2, int(os.environ.get("MMF_PIPE_SLOTS", "3")))
        self.slots = [{k: torch.empty(sh, dtype=dt, device=d) for k, (sh, dt) in shapes.items()} for _ in range(self.n)]
        self.outs = [eng.alloc_outputs(B) for _ in range(self.n)]
        self.host_out = [{k: torch.empty(v.shape, dtype=v.dtype).pin_memory() for k, v in o.items()}
                         for o in self.outs]
        self.copy_stream = torch.cuda.Stream(device=d)
        self.ready = [torch.cuda.Event() for _ in range(self.n)]
        self.free = [torch.cuda.Event() for _ in range(self.n)]
        self.done = [torch.cuda.Event() for _ in range(self.n)]
        self.i = 0

    def submit(self, batch: Dict[str, torch.Tensor]) -> int:
        """Queue one host batch {rid, rm, cid, cm, img}; returns the slot whose results
        `result(slot)` returns once the batch has finished.  Never blocks on the device except
        when the slot is still in use by the batch submitted `n` calls earlier."""
        k = self.i % self.n
        main = torch.cuda.current_stream(self.eng.device)
        if self.i >= self.n:
            self.done[k].synchronize()  # the host copy of that slot's previous results is complete
        with torch.cuda.stream(self.copy_stream):
            if self.i >= self.n:
                self.copy_stream.wait_event(self.free[k])  # compute of batch i-n has read the slot
            for n in self._IN:
                self.slots[k][n].copy_(batch[n], non_blocking=True)
            self.ready[k].record(self.copy_stream)
        main.wait_event(self.ready[k])
        sl = self.slots[k]
        self.eng.analyze_batch(sl["rid"], sl["rm"], sl["cid"], sl["cm"], sl["img"], out=self.outs[k])
        self.free[k].record(main)
        if self.d2h is not None:
            with torch.cuda.stream(self.d2h):
                self.d2h.wait_event(self.free[k])
                for n, v in self.outs[k].items():
                    self.host_out[k][n].copy_(v, non_blocking=True)
                self.done[k].record(self.d2h)
        else:
            for n, v in self.outs[k].items():
                self.host_out[k][n].copy_(v, non_blocking=True)
            self.done[k].record(main)
        self.i += 1
        return k

    def result(self, slot: int) -> Dict[str, torch.Tensor]:
        self.done[slot].synchronize()
        return self.host_out[slot]
