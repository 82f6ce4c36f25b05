"""Synthetic inputs for the matchers: vocabulary, KeyFrames, MapPoints.

The reference's vocabulary file (ORBvoc) and datasets are absent offline (.MISSING_LARGE_BLOBS), so
SearchForTriangulation runs on FeatureVectors from a seeded synthetic vocabulary tree (k = 10,
2 levels, random 32-byte centroids; descent exactly as TemplatedVocabulary::transform,
TemplatedVocabulary.h:1231-1272), and SearchByProjection on seeded MapPoints built around real
extracted keypoints.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _lib as L
from .frames import FeatureVector, Frame, LastFrameMapPoints, LocalMapPoints

_POP8 = np.array([bin(i).count("1") for i in range(256)], np.uint8)

# KITTI-like intrinsics (labelled synthetic) and arducam.yaml (TUM-shaped config)
KITTI_CAM = dict(fx=718.856, fy=718.856, cx=607.19, cy=185.22, bf=386.1448)
ARDUCAM_CAM = dict(fx=590.08, fy=590.08, cx=317.98, cy=241.15, bf=47.21)


def hamming_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """popcount(a_i xor b_j) for (n, 32) x (m, 32) uint8."""
    x = np.bitwise_xor(a[:, None, :], b[None, :, :])
    return _POP8[x].sum(axis=2, dtype=np.int32)


@dataclass
class Vocabulary:
    """A DBoW2 vocabulary tree: nodes in BFS order, children contiguous, node 0 = root."""

    k: int
    levels: int
    descriptors: np.ndarray   # (n_nodes, 32) uint8 (row 0 unused: root)
    first_child: np.ndarray   # int32, -1 for leaves
    n_children: np.ndarray    # int32
    weights: np.ndarray       # float32 word weight per node (> 0 for every leaf here)

    @staticmethod
    def synthetic(k: int = 10, levels: int = 2, seed: int = 0x0B0C0AB) -> "Vocabulary":
        rng = np.random.default_rng(seed)
        n_nodes = sum(k ** d for d in range(levels + 1))
        desc = rng.integers(0, 256, (n_nodes, 32), dtype=np.uint8)
        desc[0] = 0
        first = np.full(n_nodes, -1, np.int32)
        nch = np.zeros(n_nodes, np.int32)
        nxt = 1
        for node in range(n_nodes):
            depth = 0
            start, width = 0, 1
            while not (start <= node < start + width):
                start += width
                width *= k
                depth += 1
            if depth < levels:
                first[node] = nxt
                nch[node] = k
                nxt += k
        return Vocabulary(k, levels, desc, first, nch, np.ones(n_nodes, np.float32))

    def node_at_level(self, desc: np.ndarray, levelsup: int) -> np.ndarray:
        """TemplatedVocabulary::transform's nid for every descriptor (strict '<': first best)."""
        nid_level = self.levels - levelsup
        cur = np.zeros(len(desc), np.int64)
        nid = np.zeros(len(desc), np.int64)
        for level in range(1, self.levels + 1):
            best = np.full(len(desc), -1, np.int64)
            best_d = np.full(len(desc), 1 << 30, np.int64)
            for c in range(self.k):
                child = self.first_child[cur] + c
                d = _POP8[np.bitwise_xor(desc, self.descriptors[child])].sum(axis=1)
                better = d < best_d
                best_d = np.where(better, d, best_d)
                best = np.where(better, child, best)
            cur = best
            if level == nid_level:
                nid = cur.copy()
        return nid

    def feature_vector(self, desc: np.ndarray, levelsup: int) -> FeatureVector:
        return FeatureVector.from_assignment(self.node_at_level(desc, levelsup))


def skew(t: np.ndarray) -> np.ndarray:
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]], np.float64)


def compute_f12(tcw1: np.ndarray, tcw2: np.ndarray, K: np.ndarray) -> np.ndarray:
    """LocalMapping::ComputeF12 (LocalMapping.cc:545-561): K1^-T [t12]x R12 K2^-1."""
    R1, t1 = tcw1[:, :3].astype(np.float64), tcw1[:, 3].astype(np.float64)
    R2, t2 = tcw2[:, :3].astype(np.float64), tcw2[:, 3].astype(np.float64)
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    Kd = K.astype(np.float64)
    return (np.linalg.inv(Kd).T @ skew(t12) @ R12 @ np.linalg.inv(Kd)).astype(np.float32)


def intrinsics(cam: dict) -> np.ndarray:
    return np.array([[cam["fx"], 0, cam["cx"]], [0, cam["fy"], cam["cy"]], [0, 0, 1]], np.float32)


def pose(tx=0.0, ty=0.0, tz=0.0, yaw=0.0) -> np.ndarray:
    c, s = np.cos(yaw), np.sin(yaw)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float32)
    return np.hstack([R, np.array([[tx], [ty], [tz]], np.float32)]).astype(np.float32)


def make_frame(kps: np.ndarray, desc: np.ndarray, scale: np.ndarray, sigma2: np.ndarray,
               rows: int, cols: int, cam: dict, rng: np.random.Generator,
               stereo_frac: float = 0.5, mp_frac: float = 0.3, observed_frac: float = 0.7,
               tcw: Optional[np.ndarray] = None, u_right: Optional[np.ndarray] = None) -> Frame:
    n = len(kps)
    if u_right is None:
        disp = rng.uniform(2.0, 40.0, n).astype(np.float32)
        u_right = np.where(rng.random(n) < stereo_frac, kps["x"] - disp, -1.0).astype(np.float32)
    mp = np.zeros(n, np.uint8)
    has = rng.random(n) < mp_frac
    mp[has] = np.where(rng.random(int(has.sum())) < observed_frac, L.ORBFE_MP_OBSERVED,
                       L.ORBFE_MP_PRESENT)
    return Frame(keys_un=kps, descriptors=desc if desc is not None else np.zeros((0, 32), np.uint8),
                 u_right=u_right, mp_state=mp, scale_factors=scale, level_sigma2=sigma2,
                 min_x=0.0, max_x=float(cols), min_y=0.0, max_y=float(rows),
                 tcw=tcw, **cam)


def flip_bits(desc: np.ndarray, nflips: np.ndarray, rng: np.random.Generator) -> np.ndarray:
    out = desc.copy()
    bits = np.unpackbits(out, axis=1, bitorder="little")
    for i, k in enumerate(nflips):
        if k:
            idx = rng.choice(256, int(k), replace=False)
            bits[i, idx] ^= 1
    return np.packbits(bits, axis=1, bitorder="little")


def make_local_mappoints(F: Frame, m: int, rng: np.random.Generator, match_frac: float = 0.3,
                         max_flips: int = 40, nlevels: int = 8) -> LocalMapPoints:
    """C5-style MapPoints: uniform projections; `match_frac` of them copy a nearby
    keypoint's descriptor with up to `max_flips` random bit flips."""
    n = F.N
    px = rng.uniform(F.min_x, F.max_x, m).astype(np.float32)
    py = rng.uniform(F.min_y, F.max_y, m).astype(np.float32)
    level = rng.integers(0, nlevels, m).astype(np.int32)
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    sel = np.nonzero(rng.random(m) < match_frac)[0]
    if n and len(sel):
        src = rng.integers(0, n, len(sel))
        px[sel] = F.keys_un["x"][src] + rng.normal(0, 1.5, len(sel)).astype(np.float32)
        py[sel] = F.keys_un["y"][src] + rng.normal(0, 1.5, len(sel)).astype(np.float32)
        level[sel] = np.clip(F.keys_un["octave"][src] + rng.integers(0, 2, len(sel)), 0, nlevels - 1)
        desc[sel] = flip_bits(F.descriptors[src], rng.integers(0, max_flips + 1, len(sel)), rng)
    z = rng.uniform(0.5, 8.0, m).astype(np.float32)
    pxr = (px - np.float32(F.bf) / z).astype(np.float32)
    vc = rng.uniform(0.5, 1.0, m).astype(np.float32)
    vc[rng.random(m) < 0.1] = np.float32(0.9985)
    flags = np.full(m, L.MPF_TRACK_IN_VIEW | L.MPF_OBSERVED, np.uint8)
    flags[rng.random(m) < 0.05] &= ~np.uint8(L.MPF_TRACK_IN_VIEW)
    flags[rng.random(m) < 0.03] |= np.uint8(L.MPF_BAD)
    flags[rng.random(m) < 0.1] &= ~np.uint8(L.MPF_OBSERVED)
    return LocalMapPoints(flags, px, py, pxr, level, vc, desc)


def make_local_map(C: Frame, m: int, rng: np.random.Generator, match_frac: float = 0.5,
                   max_flips: int = 30) -> "MapPointGeometry":
    """Local-map MapPoints for isInFrustum + SearchByProjection (Tracking.cc:1186-1213): most lie
    in front of C near one of its keypoints, with MapPoint::UpdateNormalAndDepth-style distance
    bounds (MapPoint.cc:376-400) around C's keypoint level; the rest fail each isInFrustum test
    (behind the camera, outside the image, outside the scale-invariance range, oblique normal)."""
    from .frames import MapPointGeometry
    K = C.N
    Rcw = C.tcw[:, :3].astype(np.float64)
    tcw = C.tcw[:, 3].astype(np.float64)
    Ow = -Rcw.T @ tcw
    src = rng.integers(0, max(K, 1), m)
    z = rng.uniform(1.0, 30.0, m)
    u = (C.keys_un["x"][src] if K else rng.uniform(C.min_x, C.max_x, m)) + rng.normal(0, 1.0, m)
    v = (C.keys_un["y"][src] if K else rng.uniform(C.min_y, C.max_y, m)) + rng.normal(0, 1.0, m)
    kind = rng.random(m)
    u[kind < 0.05] = rng.uniform(-200, -10, int((kind < 0.05).sum()))  # outside the image
    pc = np.stack([(u - C.cx) / C.fx * z, (v - C.cy) / C.fy * z, z], axis=1)
    behind = (kind >= 0.05) & (kind < 0.08)
    pc[behind] *= -1.0
    pw = (Rcw.T @ (pc - tcw).T).T
    dist = np.linalg.norm(pw - Ow, axis=1)
    oct_ = C.keys_un["octave"][src] if K else np.zeros(m, np.int32)
    sf = np.float64(C.scale_factors[1]) if len(C.scale_factors) > 1 else 1.2
    nl = len(C.scale_factors)
    maxd = dist * sf ** (oct_ + rng.uniform(-0.45, 0.45, m))
    far = (kind >= 0.08) & (kind < 0.12)
    maxd[far] = dist[far] / 1.5                 # dist > 1.2 * mfMaxDistance
    mind = maxd / np.float64(C.scale_factors[nl - 1])
    near = (kind >= 0.12) & (kind < 0.15)
    mind[near] = dist[near] * 1.5               # dist < 0.8 * mfMinDistance
    nrm = (pw - Ow) / dist[:, None]
    nrm += rng.normal(0, 0.1, nrm.shape)
    oblique = (kind >= 0.15) & (kind < 0.2)
    nrm[oblique] = -nrm[oblique]
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    sel = np.nonzero(rng.random(m) < match_frac)[0]
    if K and len(sel):
        desc[sel] = flip_bits(C.descriptors[src[sel]], rng.integers(0, max_flips + 1, len(sel)), rng)
    flags = np.full(m, L.MPF_OBSERVED, np.uint8)
    flags[rng.random(m) < 0.05] |= np.uint8(L.MPF_BAD)
    flags[rng.random(m) < 0.1] |= np.uint8(L.MPF_SEEN)
    flags[rng.random(m) < 0.2] &= ~np.uint8(L.MPF_OBSERVED)
    flags[rng.random(m) < 0.3] |= np.uint8(L.MPF_TRACK_IN_VIEW)  # stale: isInFrustum resets it
    return MapPointGeometry(flags, pw.astype(np.float32), nrm.astype(np.float32),
                            mind.astype(np.float32), maxd.astype(np.float32), desc)


def make_lastframe(C: Frame, n: int, rng: np.random.Generator, motion: np.ndarray,
                   match_frac: float = 0.6, max_flips: int = 30) -> LastFrameMapPoints:
    """Last-frame MapPoints that re-project near current keypoints after a small motion."""
    K = C.N
    tl = pose()  # last frame at the world origin
    Rcw = C.tcw[:, :3].astype(np.float64)
    tcw = C.tcw[:, 3].astype(np.float64)
    src = rng.integers(0, max(K, 1), n)
    z = rng.uniform(2.0, 20.0, n)
    u = C.keys_un["x"][src] + rng.normal(0, 1.0, n)
    v = C.keys_un["y"][src] + rng.normal(0, 1.0, n)
    pc = np.stack([(u - C.cx) / C.fx * z, (v - C.cy) / C.fy * z, z], axis=1)
    pw = (Rcw.T @ (pc - tcw).T).T.astype(np.float32)  # world point seen at (u, v) by C
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sel = np.nonzero(rng.random(n) < match_frac)[0]
    if K and len(sel):
        desc[sel] = flip_bits(C.descriptors[src[sel]], rng.integers(0, max_flips + 1, len(sel)), rng)
    octave = np.clip(C.keys_un["octave"][src] + rng.integers(-1, 2, n), 0, len(C.scale_factors) - 1)
    angle = (C.keys_un["angle"][src] + rng.normal(0, 3.0, n)).astype(np.float32) % np.float32(360)
    wild = rng.random(n) < 0.15
    angle[wild] = rng.uniform(0, 360, int(wild.sum())).astype(np.float32)
    flags = np.full(n, L.MPF_PRESENT | L.MPF_OBSERVED, np.uint8)
    flags[rng.random(n) < 0.1] = 0
    flags[rng.random(n) < 0.05] |= np.uint8(L.MPF_OUTLIER)
    flags[rng.random(n) < 0.2] &= ~np.uint8(L.MPF_OBSERVED)
    return LastFrameMapPoints(flags, pw, desc, octave.astype(np.int32), angle, tl)
