"""Shared helpers of the parity tests (GPU path vs CPU oracle)."""
import numpy as np


def mismatch(a, b):
    """Element mask of bitwise differences; any NaN equals any NaN (NaN
    payloads/signs differ between x86 and gfx950 and carry no meaning)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype.kind == "f":
        return (a.view(np.uint32) != b.view(np.uint32)) & ~(np.isnan(a) & np.isnan(b))
    return a != b


def assert_bit_exact(gpu, ref, what):
    bad = mismatch(gpu, ref)
    if bad.any():
        idx = np.argwhere(bad)[:5]
        raise AssertionError(
            f"{what}: {bad.sum()} / {bad.size} elements differ ({bad.mean():.4%}); first at {idx.tolist()}: "
            f"gpu={np.asarray(gpu)[tuple(idx[0])]} ref={np.asarray(ref)[tuple(idx[0])]}")


def rel_depth_agreement(gpu_planes, ref_planes, costs, tol=1e-3):
    """T3 metric: fraction of pixels with cost < 2 whose depth and normal agree
    within `tol` relative."""
    d1, d2 = gpu_planes[..., 3], ref_planes[..., 3]
    m = np.isfinite(costs) & (costs < 2)
    rel = np.abs(d1 - d2) / np.maximum(np.abs(d2), 1e-12)
    n_err = np.abs(gpu_planes[..., :3] - ref_planes[..., :3]).max(axis=-1)
    ok = (rel <= tol) & (n_err <= tol)
    return float(ok[m].mean()) if m.any() else 1.0


def dmb_tree_diffs(folder_a, folder_b, views, names=("depths", "depths_geom", "normals", "costs")):
    """Every (view, map) whose .dmb differs byte-wise between two output
    trees, with the number of differing elements and the first one's
    (row, col): all of them, so a failure shows which view and pass
    diverged first instead of stopping at the first file."""
    import os
    from acmmp_amd import io as aio
    out = []
    for v in views:
        for name in names:
            pa = os.path.join(aio.result_folder(folder_a, v), name + ".dmb")
            pb = os.path.join(aio.result_folder(folder_b, v), name + ".dmb")
            with open(pa, "rb") as fa, open(pb, "rb") as fb:
                if fa.read() == fb.read():
                    continue
            a, b = aio.read_dmb(pa), aio.read_dmb(pb)
            if a.shape != b.shape:
                out.append((v, name, f"shape {a.shape} vs {b.shape}"))
                continue
            bad = mismatch(a, b)
            first = np.argwhere(bad)[0].tolist() if bad.any() else None
            out.append((v, name, f"{int(bad.sum())} elements differ, first at {first}"))
    return out


def assert_dmb_trees_equal(folder_a, folder_b, views, what, names=("depths", "depths_geom", "normals", "costs")):
    diffs = dmb_tree_diffs(folder_a, folder_b, views, names)
    if diffs:
        lines = "\n".join(f"  view {v} {n}: {d}" for v, n, d in diffs)
        raise AssertionError(f"{what}: {len(diffs)} of {len(views) * len(names)} maps differ:\n{lines}")
