"""NpyTable format and the sequence-packing loader, CPU only.

Golden vectors: tests/golden/packing.{json,npz}, produced by running the reference's
owl_wms/data/{npy_table,latent_seq_packing}.py (tests/golden/make_golden_packing.py).
Bit-exact bar: packing is index work, so slices, sample arrays and doc_id must be identical."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import ref_packing as O
from owl_wms.data import get_loader
from owl_wms.data.latent_seq_packing import (AutoEpochDistributedSampler, WindowedViewDataset, collate_fn,
                                             pack_windows)
from owl_wms.data.npy_table import NpyTable

GOLD = os.path.join(REPO, "tests", "golden")
COLS = ["depth_latent", "mouse", "buttons"]


def _gold():
    return json.load(open(os.path.join(GOLD, "packing.json"))), np.load(os.path.join(GOLD, "packing.npz"))


def _as_lists(seg, ptr):
    return [[list(map(int, r)) for r in seg[ptr[w]:ptr[w + 1]]] for w in range(len(ptr) - 1)]


def test_oracle_matches_reference_slices():
    g, _ = _gold()
    for case in g["slices"]:
        got = O.window_slices(case["lens"], case["perm"], case["window"])
        assert [[list(s) for s in w] for w in got] == case["slices"]


def test_pack_windows_matches_reference_slices():
    g, _ = _gold()
    for case in g["slices"]:
        lens = np.asarray(case["lens"])[np.asarray(case["perm"], dtype=np.int64)]
        assert _as_lists(*pack_windows(lens, case["window"])) == case["slices"]


@pytest.mark.parametrize("seed", range(20))
def test_pack_windows_matches_oracle_random(seed):
    rs = np.random.RandomState(seed)
    n = rs.randint(1, 200)
    lens = rs.randint(1, rs.choice([3, 50, 4000]), size=n)
    window = int(rs.choice([1, 7, 64, 1536]))
    perm = rs.permutation(n)
    seg, ptr = pack_windows(lens[perm], window)
    assert _as_lists(seg, ptr) == [[list(s) for s in w] for w in O.window_slices(lens, perm, window)]
    # every kept window is exactly full; windows tile the stream prefix
    assert ((np.add.reduceat(seg[:, 2] - seg[:, 1], ptr[:-1]) == window).all() if len(ptr) > 1 else True)
    assert len(ptr) - 1 == lens.sum() // window


def test_pack_windows_edge_cases():
    seg, ptr = pack_windows([], 4)
    assert seg.shape == (0, 3) and list(ptr) == [0]
    seg, ptr = pack_windows([3], 4)
    assert len(ptr) == 1
    with pytest.raises(ValueError):
        pack_windows([2, 0, 3], 4)


def _write_table(d, g, arrs, writer=NpyTable):
    t = g["table"]
    cols = COLS + ["tarball", "pt_idx", "missing", "truncated", "seq_len"]
    tbl = writer(d, columns=cols, array_columns=COLS)
    for i, n in enumerate(t["lens"]):
        tbl.append(**{k: arrs[f"row{i}_{k}"] for k in COLS}, tarball=f"shard_{i // 3}.tar", pt_idx=i,
                   missing=t["missing"][i], truncated=t["truncated"][i], seq_len=n)
    return tbl


def test_npytable_format_matches_reference(tmp_path):
    g, arrs = _gold()
    tbl = _write_table(str(tmp_path), g, arrs)
    assert (tmp_path / "schema.json").read_text() == g["table"]["schema_json"]
    assert (tmp_path / "manifest.json").read_text() == g["table"]["manifest_json"]
    # reopen: schema is read back, arrays come back memory-mapped and equal
    re = NpyTable(str(tmp_path))
    assert re.columns == tbl.columns and len(re) == len(g["table"]["lens"])
    for i in range(len(re)):
        for k in COLS:
            a = re.get([k], rows=[i])[0][0]
            assert isinstance(a, np.memmap)
            np.testing.assert_array_equal(a, arrs[f"row{i}_{k}"])
    assert re["seq_len"] == g["table"]["lens"]
    with pytest.raises(AssertionError):
        NpyTable(str(tmp_path), columns=["video"])
    with pytest.raises(ValueError):
        re.append(video=np.zeros(3))
    with pytest.raises(KeyError):
        re.get(["nope"])


@pytest.mark.parametrize("tag,epoch", [("e0", None), ("e3", 3)])
def test_packed_samples_match_reference(tmp_path, tag, epoch):
    g, arrs = _gold()
    _write_table(str(tmp_path), g, arrs)
    ds = WindowedViewDataset(str(tmp_path), g["table"]["window"], array_columns=COLS, verbose=False)
    if epoch is not None:
        ds.set_epoch(epoch)
    assert len(ds) == g["table"]["n_samples"][tag]
    for j in range(len(ds)):
        s = ds[j]
        for k in COLS + ["doc_id"]:
            ref = arrs[f"{tag}_{j}_{k}"]
            assert s[k].dtype == torch.from_numpy(ref).dtype
            np.testing.assert_array_equal(s[k].numpy(), ref)
        # the oracle's __getitem__ agrees too
        rows = [{k: arrs[f"row{i}_{k}"] for k in COLS} for i in range(len(g["table"]["lens"]))]
        o = O.sample(rows, ds._row_lookup, ds.window_slices(j), COLS)
        for k in COLS + ["doc_id"]:
            np.testing.assert_array_equal(s[k].numpy(), o[k])


def test_filters_missing_and_truncated(tmp_path):
    g, arrs = _gold()
    _write_table(str(tmp_path), g, arrs)
    t = g["table"]
    ds = WindowedViewDataset(str(tmp_path), 2, include_truncated=False, array_columns=COLS, verbose=False)
    keep = [i for i in range(len(t["lens"])) if not t["missing"][i] and not t["truncated"][i]]
    assert list(ds._row_lookup) == keep
    assert len(ds) == sum(t["lens"][i] for i in keep) // 2
    ds = WindowedViewDataset(str(tmp_path), 2, include_missing_features=True, array_columns=COLS, verbose=False)
    assert len(ds._row_lookup) == len(t["lens"])


def test_collate_and_loader(tmp_path):
    g, arrs = _gold()
    _write_table(str(tmp_path), g, arrs)
    ds = WindowedViewDataset(str(tmp_path), 4, array_columns=COLS, verbose=False)
    vid, mouse, btn, doc = collate_fn([ds[0]], COLS)
    assert vid.dtype == torch.bfloat16 and mouse.dtype == torch.bfloat16 and btn.dtype == torch.bfloat16
    assert doc.dtype == torch.int64 and vid.shape == (1, 4, 4, 2, 2) and doc.shape == (1, 4)
    loader = get_loader("sequence_packing", 1, dataset_path=str(tmp_path), window_length=4, batch_columns=COLS,
                        num_workers=0)
    seen = [b for b in loader]
    assert len(seen) == len(ds)
    with pytest.raises(AssertionError):
        get_loader("sequence_packing", 2, dataset_path=str(tmp_path), window_length=4, batch_columns=COLS)


def test_distributed_sampler_partitions_and_reshuffles():
    n = 37

    class _DS:
        def __len__(self):
            return n

    s = [AutoEpochDistributedSampler(_DS(), num_replicas=2, rank=r, shuffle=True) for r in range(2)]
    e0 = [list(x) for x in s]
    e1 = [list(x) for x in s]
    for e in (e0, e1):
        assert len(e[0]) == len(e[1]) == (n + 1) // 2
        assert set(e[0]) | set(e[1]) == set(range(n))
    assert e0 != e1  # a new permutation each iteration (latent_seq_packing.py:21-25)
