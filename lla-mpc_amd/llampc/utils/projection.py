"""Point-to-segment projection (reference: llampc/utils/projection.py:11-38).

The foot point is kept when it lies strictly inside the segment; otherwise the nearer
end vertex is returned.  ``project_segments`` does all segments of a polyline at once."""
import numpy as np


def Projection(point, line):
    assert len(point) == 1
    assert len(line) == 2
    p = np.asarray(point[0], dtype=np.float64)
    a = np.asarray(line[0], dtype=np.float64)
    b = np.asarray(line[-1], dtype=np.float64)
    proj, dist = project_segments(p, a[:, None], b[:, None])
    return proj[:, 0], float(dist[0])


def project_segments(p, A, B):
    """p [2]; A, B [2, m] segment ends -> (proj [2, m], dist [m])."""
    d = B - A
    d = d / np.linalg.norm(d, axis=0)
    t = ((p[:, None] - A) * d).sum(axis=0)
    proj = A + d * t
    ea, eb = proj - A, proj - B
    na, nb = np.linalg.norm(ea, axis=0), np.linalg.norm(eb, axis=0)
    inner = (na > 0) & (nb > 0)
    with np.errstate(invalid="ignore", divide="ignore"):
        same_dir = np.linalg.norm(ea / na - eb / nb, axis=0) <= 1e-10   # foot outside
    outside = inner & same_dir
    nearA = np.linalg.norm(A - proj, axis=0) < np.linalg.norm(B - proj, axis=0)
    proj = np.where(outside & nearA, A, np.where(outside & ~nearA, B, proj))
    return proj, np.linalg.norm(p[:, None] - proj, axis=0)
