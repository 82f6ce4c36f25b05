/*
 * orbfe_vocab.h -- DBoW2 vocabulary descent to FeatureVector on the GPU (liborbfe.so).
 *
 * Replaces TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
 * (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1140-1207, 1231-1272) for the FeatureVector half
 * consumed by ORBmatcher::SearchForTriangulation (called from KeyFrame::ComputeBoW,
 * KeyFrame.cc:59-68, with levelsup = 4). The BowVector (word weights) is not produced.
 *
 * The tree is given in DBoW2's own layout: nodes in creation (BFS) order, node 0 the root, the
 * children of a node contiguous; n_children == 0 marks a leaf (word); weights per node (a word
 * with weight 0 is stopped and skipped, :1171).
 */
#ifndef ORBFE_VOCAB_H
#define ORBFE_VOCAB_H
#include <stddef.h>
#include <stdint.h>
#include "orbfe.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orbfe_vocabulary orbfe_vocabulary;

/* levels = m_L (depth of the tree). node_desc: n_nodes x 32 bytes. */
int orbfe_vocab_create(int n_nodes, int levels, const uint8_t* node_desc,
                       const int32_t* first_child, const int32_t* n_children,
                       const float* weights, int device, orbfe_vocabulary** out);
int orbfe_vocab_destroy(orbfe_vocabulary* v);

/* FeatureVector of n descriptors (host memory) as CSR: node_ids[*n_nodes], offsets[*n_nodes+1],
 * indices[offsets[*n_nodes]]; buffers sized n (offsets n + 1). n <= 8192. */
int orbfe_vocab_transform(orbfe_vocabulary* v, const uint8_t* desc, int n, int levelsup,
                          uint32_t* node_ids, int32_t* offsets, int32_t* indices, int* n_nodes);

/* Device batch: image i has d_counts[i] descriptors at d_desc + i*desc_stride; its CSR goes to
 * d_node_ids + i*cap, d_offsets + i*(cap+1), d_indices + i*cap, d_n_nodes[i]. cap <= 8192. */
int orbfe_vocab_transform_batch_device(orbfe_vocabulary* v, int n_images, const uint8_t* d_desc,
                                       size_t desc_stride, const int32_t* d_counts, int levelsup,
                                       uint32_t* d_node_ids, int32_t* d_offsets,
                                       int32_t* d_indices, int32_t* d_n_nodes, int cap,
                                       void* stream);
#ifdef __cplusplus
}
#endif
#endif
