"""The native extension builds for gfx950 (hipcc cross-compiles without a GPU) and imports."""
from pytorch_mnist_ddp_amd import _build


def test_build_is_incremental_and_importable():
    out = _build.build()
    from pytorch_mnist_ddp_amd.ops import native
    C = native.load(build_if_missing=False)
    assert C.PARAM_TOTAL == 1200000 and C.FC1_KSPLIT == 32
    offs = C.PARAM_OFFSETS
    assert all(v % 64 == 0 for v in offs.values())
    assert C.BUCKET_SPLIT == offs["conv1.weight"]
    # the shared object carries gfx950 code objects only
    blob = open(out, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"amdgcn-amd-amdhsa--gfx942" not in blob and b"amdgcn-amd-amdhsa--gfx90a" not in blob
    assert out.endswith(".so")
