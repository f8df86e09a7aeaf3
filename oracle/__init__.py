"""ORACLE — test infrastructure, not product code.

A CPU (PyTorch fp32) restatement of the reference's MisinfoForensics.analyze() 5-signal path,
used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
and as the timed CPU baseline ("kind": "port").  The product path (mmf_amd) never imports it.

Pinning: tests/golden/make_golden.py drives the reference code itself (imported from
/root/reference in the build container with `dotenv`/`torchvision` stubs) on the same
synthetic weights/inputs and commits the outputs under tests/golden/; tests/test_oracle.py
checks this restatement against them.  EfficientNet-B0 (torchvision absent) is proxy-pinned
against transformers' independent EfficientNet configured as B0 (tests/test_oracle_effnet_hf.py).
The host-input restatements are pinned to Pillow itself, the library the reference calls:
pil_resample.py (tests/test_pil_resample_cpu.py) and jpeg_decode.py (tests/test_jpeg_cpu.py),
bit for bit.
"""
