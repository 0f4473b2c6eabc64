"""scan_octrees / generate_points (kaolin/ops/spc/spc.py:40-98) over the HIP path."""
from ... import _C


def scan_octrees(octrees, lengths):
    r"""-> (max_level, pyramids (B,2,L+2) CPU int32, exsum (num_bytes + B) int32)."""
    return _C.ops.spc.scan_octrees_cuda(octrees.contiguous(), lengths.contiguous())


def generate_points(octrees, pyramids, exsum):
    r"""Point hierarchies (num_points_all_levels, 3) int16 of a batch of octrees."""
    return _C.ops.spc.generate_points_cuda(octrees.contiguous(), pyramids.contiguous(), exsum.contiguous())
