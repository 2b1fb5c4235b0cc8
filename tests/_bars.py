"""The suite's fp32 parity bar (test infrastructure, CPU-only helpers shared by every suite).

    elementwise:  max_e |got - ref| / max(|ref_e|, 1e-3 · max|ref|)   <= 1e-4
    normwise:     ||got - ref||_2 / ||ref||_2                          <= 1e-4
Where the elementwise bar fails against the fp32 reference (two fp32 summation orders that
differ at a cancellation), the check is decided against the float64 truth: the result must be
within max(1e-4, factor × the fp32 reference's own error against that truth)."""
import torch

TOL = 1e-4
FLOOR = 1e-3


def max_rel_err(got, ref, floor=FLOOR) -> float:
    """max_e |got - ref| / max(|ref_e|, floor·max|ref|)  (0 for empty / all-zero ref and got)."""
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    if ref.numel() == 0:
        return 0.0
    err = (got - ref).abs()
    scale = float(ref.abs().max())
    if scale == 0.0:
        return float("inf") if float(err.max()) > 0 else 0.0
    return float((err / ref.abs().clamp_min(floor * scale)).max())


def normwise_err(got, ref) -> float:
    """||got - ref||_2 / ||ref||_2 over the whole tensor (0 for an all-zero pair)."""
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    if not bool(torch.isfinite(ref).all()):
        m = torch.isfinite(ref)
        got, ref = got[m], ref[m]
    den = float(ref.norm())
    num = float((got - ref).norm())
    return num / den if den > 0 else (0.0 if num == 0 else float("inf"))


def passes(got, ref32, ref64=None, factor=2.0, tol=TOL) -> tuple[bool, str]:
    """(ok, message) of the bar above."""
    nw = normwise_err(got, ref32)
    e = max_rel_err(got, ref32)
    if nw > tol:
        return False, f"normwise {nw:.3e} > {tol:.0e}"
    if e <= tol:
        return True, ""
    if ref64 is None:
        return False, f"elementwise {e:.3e} > {tol:.0e} (no float64 truth)"
    eg, ec = max_rel_err(got, ref64), max_rel_err(ref32, ref64)
    ok = eg <= max(tol, factor * ec)
    return ok, f"elementwise {e:.3e}; vs float64 {eg:.3e}, fp32 reference {ec:.3e} (x{factor})"
