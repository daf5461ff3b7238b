"""On-disk / wire formats and sub-SVO linking, CPU only.

* CompactSVO.SaveToDisk (CompactSVO.cs:80-86): raw little-endian int32
  descriptors, no header, no attachments;
* the reference's `Text` debug dump (Assets/Scripts/SVO/CompactSVO/Text):
  parsed by the product importer and compared with the committed fixture;
* the native SVOP pool file (header + nodes + attachments);
* NaiveCreator.Create(root, getLeaf) linking (NaiveCreator.cs:30-42,156-159;
  Clipmap.cs:153-169): the product's link_leaves against the object-recursive
  restatement in oracle/naive_creator.py, bit for bit.
"""
import os

import numpy as np
import pytest

from raytracingtest_amd.builder import build_menger, link_leaves
from raytracingtest_amd.svo_data import SVOData, SVOFormatError

TEXT_DUMP = "/root/reference/Assets/Scripts/SVO/CompactSVO/Text"


def test_int32_dump_roundtrip_is_raw_little_endian(tmp_path, text_svo):
    p = tmp_path / "svo.bin"
    text_svo.save_int32_dump(str(p))
    raw = p.read_bytes()
    assert len(raw) == 4 * len(text_svo)                       # no header, no attachments
    assert raw == text_svo.childDescriptors.astype("<i4").tobytes()
    back = SVOData.load_int32_dump(str(p))
    assert np.array_equal(back.childDescriptors, text_svo.childDescriptors)
    assert not back.attachments.any()                          # SaveToDisk drops them
    # a V2-only pool cannot be written in the 16-bit reference format
    wide = build_menger(8)
    assert wide.format == 2
    with pytest.raises(SVOFormatError):
        wide.save_int32_dump(str(tmp_path / "wide.bin"))


@pytest.mark.parametrize("kind", ["v1", "v2"])
def test_svop_roundtrip(tmp_path, text_svo, kind):
    svo = text_svo if kind == "v1" else build_menger(6).as_v2()
    assert svo.format == (1 if kind == "v1" else 2)
    p = str(tmp_path / "pool.svop")
    svo.save(p)
    back = SVOData.load(p)
    assert back.format == svo.format and len(back) == len(svo)
    assert np.array_equal(back.to_v2(), svo.to_v2())
    assert np.array_equal(back.attachments, svo.attachments)
    size = os.path.getsize(p)
    assert size == 20 + (4 if kind == "v1" else 8) * len(svo) + 8 * len(svo)


def test_svop_rejects_bad_files(tmp_path, text_svo):
    p = tmp_path / "pool.svop"
    text_svo.save(str(p))
    raw = p.read_bytes()
    (tmp_path / "trunc.svop").write_bytes(raw[:-5])
    with pytest.raises(SVOFormatError):
        SVOData.load(str(tmp_path / "trunc.svop"))
    (tmp_path / "magic.svop").write_bytes(b"XXXX" + raw[4:])
    with pytest.raises(SVOFormatError):
        SVOData.load(str(tmp_path / "magic.svop"))
    (tmp_path / "ver.svop").write_bytes(raw[:4] + (99).to_bytes(4, "little") + raw[8:])
    with pytest.raises(SVOFormatError):
        SVOData.load(str(tmp_path / "ver.svop"))


@pytest.mark.skipif(not os.path.exists(TEXT_DUMP), reason="reference Text dump not present")
def test_parse_text_dump_matches_fixture(text_fixture, text_svo):
    """The product importer reads the reference's own file to the same pool as
    the committed fixture (tests/golden/make_text_fixture.py)."""
    svo = SVOData.parse_text_dump(TEXT_DUMP)
    assert len(svo) == 4977 and svo.format == 1
    assert np.array_equal(svo.to_v2(), text_svo.to_v2())
    assert np.array_equal(svo.attachments, text_svo.attachments)
    assert svo.depth() == 6 and len(svo.leaf_voxels()) == 10464


def test_parse_text_dump_rejects_garbage(tmp_path):
    p = tmp_path / "Text"
    p.write_text("header\nCD: [ChildDescriptor childPointer: 1, validMask: 0000000x]\n")
    with pytest.raises(SVOFormatError):
        SVOData.parse_text_dump(str(p))


def _target(ix, iy, iz, level):
    # several link targets, so "the last leaf child wins" is exercised
    return 10000 + (ix * 7 + iy * 3 + iz) % 5


@pytest.mark.parametrize("get_leaf", [lambda *a: 10000, _target], ids=["clipmap_const", "varying"])
def test_link_leaves_matches_naive_creator_restatement(get_leaf):
    """The product's link_leaves on an unlinked Custom1 pool (maxLevel 5) equals
    NaiveCreator.Create(root, getLeaf) as restated object-recursively."""
    from oracle import naive_creator as nc
    desc, att = nc.create(4, 5)
    plain = SVOData(childDescriptors=desc, attachments=att)
    want_desc, want_att = nc.create(4, 5, get_leaf=get_leaf)
    got = link_leaves(plain, get_leaf)
    assert got.format == 1
    assert np.array_equal(got.childDescriptors, want_desc)
    assert np.array_equal(got.attachments, want_att)
    # every former leaf is now a valid non-leaf slot; nothing else changed
    lo0, _ = plain.masks_and_first()
    lo1, first1 = got.masks_and_first()
    linked = (lo0 & 0xFF) != ((lo0 >> 8) & 0xFF)
    assert np.all((lo1 & 0xFF)[linked] == (lo1 >> 8)[linked] & 0xFF)
    assert np.all(first1[linked] >= 10000)


def test_link_leaves_rejects_mixed_nodes():
    # root: slot 0 a non-leaf child (node 1), slot 1 a leaf
    nodes = np.array([(1 << 32) | (0x03 << 8) | 0x01, (0x01 << 8)], np.uint64)
    svo = SVOData(nodes=nodes)
    with pytest.raises(ValueError):
        link_leaves(svo, lambda *a: 100)
