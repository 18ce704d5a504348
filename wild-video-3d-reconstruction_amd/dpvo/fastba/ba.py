"""fastba operator surface (reference dpvo/fastba/ba.py) over the cuda_ba
drop-in (csrc/fastba.hip)."""
import cuda_ba

neighbors = cuda_ba.neighbors   # device-resident (the reference round-trips to the host)
reproject = cuda_ba.reproject


def BA(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1, iterations=2, csr=None, status=None,
       keep_status=False):
    """Gauss-Newton over poses [t0, t1) and the inverse depth of every patch
    referenced by kk; `poses` and `patches` are updated in place.  csr
    (optional): the caller's update_ops.group_by(kk) CSR, reused instead of
    grouping the edges again.  status (optional): a device int32 [1] that
    receives the Cholesky status instead of a host read (cuda_ba.forward)."""
    return cuda_ba.forward(poses.data, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1, iterations,
                           csr=csr, status=status, keep_status=keep_status)
