"""Host logic of the row-marked optimizer sweep (no GPU): FusedAdam._marks maps a launch range to the marked table's
row offset (negative when the launch starts inside the table) and skips ranges outside it; ops.row_marks_bytes is
the C ABI's layout (stamps, padding to 16 B + 16, 1 KB zero tail)."""
import types

import torch


def _opt(numel, marks):
    import rbm_amd  # noqa: F401
    from rbm_amd.train_step import FusedAdam
    flat = types.SimpleNamespace(numel=numel, device=torch.device("cpu"))
    opt = FusedAdam(flat)
    opt.marks = marks
    return opt


def test_marks_for_launch_ranges():
    rm, ep = torch.zeros(8), torch.zeros(1)
    tlo, rows, dshift = 1024, 100, 7            # table elements [1024, 1024 + 12800)
    opt = _opt(20000, (tlo, rows, dshift, rm, ep))
    assert opt._marks(0, 20000) == (rm, ep, 1024, 100, 7)          # table inside the range
    assert opt._marks(2048, 4096) == (rm, ep, -1024, 100, 7)       # range starts inside the table
    assert opt._marks(0, 1024) is None                             # ends where the table starts
    assert opt._marks(1024 + 12800, 20000) is None                 # starts where it ends
    assert opt._marks(1024 + 12796, 20000) == (rm, ep, -12796, 100, 7)
    assert _opt(20000, None)._marks(0, 20000) is None


def test_row_marks_bytes_layout():
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    for rows in (1, 15, 16, 17, 54543, 1_000_002):
        n = ops.row_marks_bytes(rows)
        zeros_at = (rows + 15) // 16 * 16 + 16
        assert zeros_at >= rows + 16 and zeros_at % 16 == 0          # scalar mark loads run <= 15 B past a row
        assert n == zeros_at + 1024                                   # the 1 KB zero tail (64 lanes x 16 B)
