"""Host logic of the load-time precision calibration (engine.py), no device: the RoBERTa precise-mode
operand masks the calibration walks (option text_prec_mask: bit k = GEMM kind k -- QKV, out-proj,
FFN-1, FFN-2 -- on hi / lo activations, bit k + 4 = also on W_lo) and the user-pin detection that
keeps a set_option / environment choice out of the calibration's hands."""
from types import SimpleNamespace

from mmf_amd.engine import Engine


def test_prec_masks_cover_every_level_cheapest_first():
    ms = Engine._prec_masks()
    # three levels per kind (fp16 operands, hi / lo activations, + W_lo) for four kinds, minus the full mode
    assert len(ms) == 3 ** 4 - 1 and len(set(ms)) == len(ms)
    assert Engine.PREC_FULL not in ms and ms[0] == 0
    for m in ms:
        assert 0 <= m < 256
        assert (m >> 4) & ~m & 15 == 0, f"mask {m}: W_lo on a kind without hi / lo activations"
    costs = [Engine._mask_cost(m) for m in ms]
    assert costs == sorted(costs)
    assert max(costs) < Engine._mask_cost(Engine.PREC_FULL)


def test_mask_cost_counts_products_per_kind():
    c = Engine.PREC_KIND_COST
    assert Engine._mask_cost(0) == sum(c)                 # one fp16 product per kind
    assert Engine._mask_cost(Engine.PREC_FULL) == 3 * sum(c)  # three products per kind
    assert Engine._mask_cost(1) == sum(c) + c[0]          # QKV on hi / lo activations: two products
    assert Engine._mask_cost(1 | 16) == sum(c) + 2 * c[0]  # ... and W_lo: three
    assert Engine._mask_cost(16) == sum(c)                # a W_lo bit without its activation bit is inert


def _stub(options):
    s = SimpleNamespace(_auto_set={}, opts=dict(options))
    s.get_option = lambda name: s.opts[name]

    def set_option(name, value):
        s.opts[name] = int(value)
    s.set_option = set_option
    return s


def test_pin_detection():
    s = _stub({"text_hilo": -1, "effnet_fp32": 0})
    assert not Engine._pinned(s, "text_hilo")       # never written by the engine: no record, no pin
    Engine._auto_write(s, "text_hilo", -1)
    assert s.opts["text_hilo"] == -1 and not Engine._pinned(s, "text_hilo")
    s.set_option("text_hilo", 1)                      # a user's set_option after the engine's write
    assert Engine._pinned(s, "text_hilo")
    Engine._auto_write(s, "text_hilo", 2)             # the engine's own later write clears it
    assert not Engine._pinned(s, "text_hilo")
    s._auto_set["effnet_fp32"] = 0
    s.set_option("effnet_fp32", 1)
    assert Engine._pinned(s, "effnet_fp32")
