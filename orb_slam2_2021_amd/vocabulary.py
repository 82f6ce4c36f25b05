"""ORBVocabulary on MI355X: the DBoW2 vocabulary (include/orbfe_vocab.h).

Mirrors TemplatedVocabulary<FORB::TDescriptor, FORB> for the per-frame path:
  loadFromTextFile / loadFromBinaryFile   (TemplatedVocabulary.h:1351-1440, 1467-1511)
  transform(features, BowVector, FeatureVector, levelsup)   (TemplatedVocabulary.h:1140-1272)
as called by Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame.cc:447-454, KeyFrame.cc:59-68).
"""
from __future__ import annotations

from ctypes import byref, c_int, c_size_t, c_void_p
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .frames import FeatureVector


@dataclass
class BowVector:
    """DBoW2::BowVector (std::map<WordId, WordValue>): word ids ascending, double weights."""

    words: np.ndarray    # uint32
    weights: np.ndarray  # float64

    def as_dict(self):
        return dict(zip(self.words.tolist(), self.weights.tolist()))


class ORBVocabulary:
    def __init__(self, handle: c_void_p):
        self._lib = L.lib()
        self._h = handle
        info = (c_int * 6)()
        L.check(self._lib.orbfe_vocab_get_info(self._h, info), "orbfe_vocab_get_info")
        (self.n_nodes, self.n_words, self.k, self.levels, self.scoring, self.weighting) = list(info)

    @staticmethod
    def from_table(k: int, levels: int, scoring: int, weighting: int, parent: np.ndarray,
                   is_leaf: np.ndarray, descriptors: np.ndarray, weights: np.ndarray,
                   device: int = 0) -> "ORBVocabulary":
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        descriptors = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        weights = np.ascontiguousarray(weights, np.float64)
        h = c_void_p()
        L.check(L.lib().orbfe_vocab_create(len(parent), int(k), int(levels), int(scoring),
                                           int(weighting), L.ptr(parent), L.ptr(is_leaf),
                                           L.ptr(descriptors), L.ptr(weights), int(device), byref(h)),
                "orbfe_vocab_create")
        return ORBVocabulary(h)

    @staticmethod
    def from_tree(tree, device: int = 0) -> "ORBVocabulary":
        """From a synthetic.Vocabulary (or anything with the same fields)."""
        return ORBVocabulary.from_table(tree.k, tree.levels, getattr(tree, "scoring", 0),
                                        getattr(tree, "weighting", 0), tree.parent, tree.is_leaf,
                                        tree.descriptors, tree.weights, device)

    @staticmethod
    def loadFromTextFile(path: str, device: int = 0) -> "ORBVocabulary":
        h = c_void_p()
        L.check(L.lib().orbfe_vocab_load_text(str(path).encode(), int(device), byref(h)),
                "orbfe_vocab_load_text")
        return ORBVocabulary(h)

    @staticmethod
    def loadFromBinaryFile(path: str, device: int = 0) -> "ORBVocabulary":
        h = c_void_p()
        L.check(L.lib().orbfe_vocab_load_binary(str(path).encode(), int(device), byref(h)),
                "orbfe_vocab_load_binary")
        return ORBVocabulary(h)

    def tables(self) -> dict:
        n = self.n_nodes
        t = {"parent": np.zeros(n, np.int32), "is_leaf": np.zeros(n, np.uint8),
             "descriptors": np.zeros((n, 32), np.uint8), "weights": np.zeros(n, np.float64),
             "word_id": np.zeros(n, np.uint32)}
        L.check(self._lib.orbfe_vocab_export(self._h, L.ptr(t["parent"]), L.ptr(t["is_leaf"]),
                                             L.ptr(t["descriptors"]), L.ptr(t["weights"]),
                                             L.ptr(t["word_id"])), "orbfe_vocab_export")
        return t

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.orbfe_vocab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def transform(self, descriptors: np.ndarray, levelsup: int = 4):
        """TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup) ->
        (BowVector, FeatureVector)."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        words = np.zeros(max(n, 1), np.uint32)
        wts = np.zeros(max(n, 1), np.float64)
        ids = np.zeros(max(n, 1), np.uint32)
        offs = np.zeros(n + 1, np.int32)
        idx = np.zeros(max(n, 1), np.int32)
        nw, nn = c_int(), c_int()
        L.check(self._lib.orbfe_vocab_transform(self._h, L.ptr(d), n, int(levelsup), L.ptr(words),
                                                L.ptr(wts), byref(nw), L.ptr(ids), L.ptr(offs),
                                                L.ptr(idx), byref(nn)), "vocab_transform")
        k = nn.value
        return (BowVector(words[:nw.value].copy(), wts[:nw.value].copy()),
                FeatureVector(ids[:k], offs[:k + 1], idx[:offs[k]]))

    def transform_batch_device(self, n_images: int, d_desc: int, desc_stride: int, d_counts: int,
                               levelsup: int, d_node_ids: int, d_offsets: int, d_indices: int,
                               d_n_nodes: int, cap: int, stream: int = 0, d_bow_words: int = 0,
                               d_bow_weights: int = 0, d_bow_n: int = 0) -> None:
        L.check(self._lib.orbfe_vocab_transform_batch_device(
            self._h, int(n_images), c_void_p(d_desc), c_size_t(desc_stride), c_void_p(d_counts),
            int(levelsup), c_void_p(d_bow_words), c_void_p(d_bow_weights), c_void_p(d_bow_n),
            c_void_p(d_node_ids), c_void_p(d_offsets), c_void_p(d_indices), c_void_p(d_n_nodes),
            int(cap), c_void_p(stream)), "vocab_transform_batch_device")
