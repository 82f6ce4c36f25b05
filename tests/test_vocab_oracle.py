"""DBoW2 vocabulary on CPU: the oracle's restatement (oracle/orbref_vocab.cpp) against an
independent numpy/Python restatement, the reference's file formats written by
synthetic.Vocabulary.save_text / save_binary (saveToTextFile / saveToBinaryFile,
TemplatedVocabulary.h:1441-1461, 1516-1537), and liborbfe's loaders (host-only, device = -1)
against the oracle's loaders. No GPU."""
import os

import numpy as np
import pytest

from orb_slam2_2021_amd import synthetic as S
from oracle.orbref import RefVocabulary


def python_transform(voc, desc, levelsup):
    """TemplatedVocabulary::transform (TemplatedVocabulary.h:1140-1207) with a dict BowVector and
    Python floats (IEEE doubles, the same rounding as WordValue)."""
    nid, leaf = voc.descend(desc, levelsup)
    w = voc.weights[leaf]
    word_of = np.cumsum(voc.is_leaf) - 1  # word ids in node order
    bow, fv = {}, {}
    additive = voc.weighting in (0, 1)
    for i in range(len(desc)):
        if not w[i] > 0:
            continue
        wid = int(word_of[leaf[i]])
        if wid in bow:
            if additive:
                bow[wid] += float(w[i])
        else:
            bow[wid] = float(w[i])
        fv.setdefault(int(nid[i]), []).append(i)
    must = voc.scoring != 5
    if additive and bow and not must:
        nd = float(len(bow))
        bow = {k: v / nd for k, v in bow.items()}
    if must:
        norm = 0.0
        for k in sorted(bow):
            norm += abs(bow[k]) if voc.scoring != 1 else bow[k] * bow[k]
        if voc.scoring == 1:
            norm = float(np.sqrt(norm))
        if norm > 0.0:
            bow = {k: v / norm for k, v in bow.items()}
    return bow, fv


def ref_of(voc):
    return RefVocabulary.from_table(voc.k, voc.levels, voc.scoring, voc.weighting, voc.parent,
                                    voc.is_leaf, voc.descriptors, voc.weights)


def descriptors(rng, voc, n):
    """Half random, half near words (a few bits off a random leaf): both kinds of descent."""
    d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    leaves = np.nonzero(voc.is_leaf)[0]
    near = voc.descriptors[rng.choice(leaves, n // 2)].copy()
    near ^= (rng.integers(0, 256, near.shape, dtype=np.uint8) & rng.integers(0, 256, near.shape, dtype=np.uint8)
             & rng.integers(0, 256, near.shape, dtype=np.uint8))
    d[: n // 2] = near
    return d


@pytest.mark.parametrize("scoring,weighting", [(0, 0), (0, 1), (1, 0), (2, 2), (5, 0), (5, 3), (1, 3)])
def test_oracle_transform_matches_python(scoring, weighting):
    rng = np.random.default_rng(scoring * 7 + weighting)
    voc = S.Vocabulary.synthetic_orbvoc(k=6, levels=4, seed=11, stop_frac=0.05, scoring=scoring,
                                        weighting=weighting)
    ref = ref_of(voc)
    for n, levelsup in [(0, 4), (1, 2), (700, 2), (700, 0), (300, 4), (300, 6)]:
        d = descriptors(rng, voc, n)
        words, weights, (ids, offs, idx) = ref.transform(d, levelsup)
        bow, fv = python_transform(voc, d, levelsup)
        assert words.tolist() == sorted(bow)
        assert weights.tolist() == [bow[k] for k in sorted(bow)]  # bit-exact doubles
        assert ids.tolist() == sorted(fv)
        assert [idx[offs[j]:offs[j + 1]].tolist() for j in range(len(ids))] == [fv[k] for k in sorted(fv)]


def test_orbvoc_shape_and_levelsup4():
    voc = S.Vocabulary.synthetic_orbvoc()
    assert voc.n_nodes == 1111111 and int(voc.is_leaf.sum()) == 10 ** 6
    rng = np.random.default_rng(3)
    d = descriptors(rng, voc, 400)
    words, weights, (ids, offs, idx) = ref_of(voc).transform(d, 4)
    bow, fv = python_transform(voc, d, 4)
    assert words.tolist() == sorted(bow) and weights.tolist() == [bow[k] for k in sorted(bow)]
    assert ids.tolist() == sorted(fv)
    # levelsup 4 of L = 6: FeatureVector nodes are level-2 nodes (ids 11..110)
    assert ids.min() >= 11 and ids.max() <= 110
    assert abs(weights.sum() - 1.0) < 1e-12  # L1-normalised


def test_text_file_round_trip(tmp_path):
    voc = S.Vocabulary.synthetic_orbvoc(k=5, levels=3, seed=2, stop_frac=0.1)
    path = tmp_path / "voc.txt"
    voc.save_text(str(path))
    ref = RefVocabulary.load(str(path))
    assert ref is not None
    info = ref.info()
    assert info == {"n_nodes": voc.n_nodes, "n_words": int(voc.is_leaf.sum()), "k": 5, "levels": 3,
                    "scoring": 0, "weighting": 0}
    t = ref.tables()
    assert np.array_equal(t["parent"][1:], voc.parent[1:])
    assert np.array_equal(t["descriptors"], voc.descriptors)
    assert np.array_equal(t["is_leaf"], voc.is_leaf)
    # the weight goes through ostream's default %g (6 significant digits)
    assert np.array_equal(t["weights"], np.array([float(f"{w:g}") for w in voc.weights]))


def test_binary_file_round_trip_appends_the_eof_copy(tmp_path):
    voc = S.Vocabulary.synthetic_orbvoc(k=4, levels=3, seed=5, stop_frac=0.1)
    path = tmp_path / "voc.bin"
    voc.save_binary(str(path))
    ref = RefVocabulary.load(str(path), binary=True)
    t = ref.tables()
    n = voc.n_nodes
    assert ref.info()["n_nodes"] == n + 1 and ref.info()["n_words"] == int(voc.is_leaf.sum()) + 1
    assert np.array_equal(t["parent"][1:n], voc.parent[1:])
    assert t["parent"][n] == voc.parent[n - 1]
    assert np.array_equal(t["descriptors"][n], voc.descriptors[n - 1])
    assert np.array_equal(t["weights"][:n], voc.weights.astype(np.float32).astype(np.float64))
    # the copy is the later sibling with the same descriptor: never strictly closer, so the
    # transform equals the transform of the table without it
    rng = np.random.default_rng(9)
    d = descriptors(rng, voc, 500)
    v32 = S.Vocabulary(voc.k, voc.levels, voc.descriptors, voc.first_child, voc.n_children,
                       voc.weights.astype(np.float32).astype(np.float64))
    a = ref.transform(d, 1)
    b = ref_of(v32).transform(d, 1)
    for x, y in zip(a[:2] + a[2], b[:2] + b[2]):
        assert np.array_equal(x, y)


def test_malformed_files_are_rejected(tmp_path):
    bad = tmp_path / "bad.txt"
    bad.write_text("10 6 9 0\n")  # scoring out of range (loadFromTextFile :1374)
    assert RefVocabulary.load(str(bad)) is None
    voc = S.Vocabulary.synthetic(k=3, levels=1)
    p = tmp_path / "v.bin"
    voc.save_binary(str(p))
    raw = p.read_bytes()
    (tmp_path / "short.bin").write_bytes(raw[:-5])
    assert RefVocabulary.load(str(tmp_path / "short.bin"), binary=True) is None


# ---- liborbfe's loaders, host-only (no device needed) ----

def lib_load(path, binary):
    from ctypes import byref, c_void_p
    from orb_slam2_2021_amd import _lib as L
    from orb_slam2_2021_amd.vocabulary import ORBVocabulary
    h = c_void_p()
    fn = L.lib().orbfe_vocab_load_binary if binary else L.lib().orbfe_vocab_load_text
    st = fn(str(path).encode(), -1, byref(h))
    return ORBVocabulary(h) if st == 0 else None


@pytest.mark.parametrize("binary", [False, True])
def test_library_loaders_match_the_oracle(tmp_path, binary):
    voc = S.Vocabulary.synthetic_orbvoc(k=7, levels=3, seed=21, stop_frac=0.05, scoring=1, weighting=1)
    path = tmp_path / ("v.bin" if binary else "v.txt")
    (voc.save_binary if binary else voc.save_text)(str(path))
    mine = lib_load(path, binary)
    ref = RefVocabulary.load(str(path), binary=binary)
    assert mine is not None and ref is not None
    assert (mine.n_nodes, mine.n_words, mine.k, mine.levels, mine.scoring, mine.weighting) == \
        tuple(ref.info()[k] for k in ("n_nodes", "n_words", "k", "levels", "scoring", "weighting"))
    a, b = mine.tables(), ref.tables()
    for key in ("parent", "is_leaf", "descriptors", "weights", "word_id"):
        assert np.array_equal(a[key], b[key]), key
    mine.close()


def test_library_loader_rejects_what_the_oracle_rejects(tmp_path):
    (tmp_path / "a.txt").write_text("21 6 0 0\n")  # k > 20
    assert lib_load(tmp_path / "a.txt", False) is None
    (tmp_path / "b.txt").write_text("10 2 0 0\n5 1 " + "0 " * 32 + "1.0\n")  # parent not yet defined
    assert lib_load(tmp_path / "b.txt", False) is None
    assert RefVocabulary.load(str(tmp_path / "b.txt")) is None
    voc = S.Vocabulary.synthetic(k=3, levels=1)
    voc.save_binary(str(tmp_path / "c.bin"))
    raw = (tmp_path / "c.bin").read_bytes()
    (tmp_path / "d.bin").write_bytes(raw + raw[-41:])  # one record too many
    assert lib_load(tmp_path / "d.bin", True) is None
    assert RefVocabulary.load(str(tmp_path / "d.bin"), binary=True) is None


def test_host_only_vocabulary_refuses_transform(tmp_path):
    from orb_slam2_2021_amd import _lib as L
    voc = S.Vocabulary.synthetic(k=3, levels=1)
    voc.save_text(str(tmp_path / "v.txt"))
    mine = lib_load(tmp_path / "v.txt", False)
    with pytest.raises(L.OrbfeError):
        mine.transform(np.zeros((4, 32), np.uint8))
