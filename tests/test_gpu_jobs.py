"""BWT job kernels on the GPU, beyond the end-to-end parity tests.

The round-4 bug: the compare-exchange inline asm wrote SCC without declaring it, and in the
2-wave job kernel a lane-mask select after one of them used the asm's SCC -- a network stage ran
in the inverted direction whenever that SCC came out zero, which depended on the keys.  It showed
as about one wrong 256 KiB block per 20 encodes of the 1024-chunk text stream (round-1 sorts of
~300-element workgroup jobs whose keys share all rotation bits), because the MSD scatter orders
a bucket's elements differently from run to run.  Re-running the job phase of one encode with
every job's inputs reordered reproduced it deterministically (10 failing jobs in 200 re-runs with
seed 1000 on the unfixed build); tests/test_isa.py checks the machine code for the pattern.
"""
import importlib

import pytest
import torch

bra = importlib.import_module("br-archive_amd")
pytestmark = pytest.mark.gpu


def test_job_sorts_on_random_keys():
    for w in (1, 2, 4):
        assert bra.sortnet_selftest(w, 8192 // w, 64, 7 * w) == 0, w


@pytest.mark.parametrize("kind,bs,nb", [(bra.SYNTH_TEXT, 256 * 1024, 1024), (bra.SYNTH_SYM16, 1 << 20, 64)],
                         ids=["text_256KiB_x1024", "sym16_1MiB_x64"])
def test_job_phase_any_input_order(kind, bs, nb):
    """Every job gives its input rotations back (and no slot belongs to two jobs) whatever order
    the MSD levels left its elements in: 200 re-runs of one encode's job phase, inputs reordered."""
    codec = bra.BlockCodec(0)
    try:
        d = torch.from_numpy(bra.synth_fill(kind, bs * nb, bs)).cuda()
        codec.encode(d, bs)
        torch.cuda.synchronize()
        assert codec.debug_rerun_jobs(20, 0) == 0  # inputs as the levels left them
        assert codec.debug_rerun_jobs(200, 1000) == 0
    finally:
        codec.close()


def test_debug_entry_points_reject_stale_or_invalid_requests():
    """the sort self-test takes 1, 2 or 4 waves only, and the job re-run refuses once a
    decode (or a fallback) has run on the context since the encode."""
    for w in (0, 3, 8, -1):
        with pytest.raises(RuntimeError):
            bra.sortnet_selftest(w, 1, 1, 1)
    codec = bra.BlockCodec(0)
    try:
        bs = 65536
        d = torch.from_numpy(bra.synth_fill(bra.SYNTH_TEXT, 4 * bs, bs)).cuda()
        with pytest.raises(RuntimeError):
            codec.debug_rerun_jobs(1)  # nothing encoded yet
        hdr, off, pay = codec.encode(d, bs)
        torch.cuda.synchronize()
        assert codec.debug_rerun_jobs(2) == 0
        out = codec.decode(hdr, off, pay, d.numel(), bs)
        assert torch.equal(out, d)
        with pytest.raises(RuntimeError):
            codec.debug_rerun_jobs(1)
    finally:
        codec.close()
