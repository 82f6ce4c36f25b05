/*
 * orbfe_vocab.h -- the DBoW2 ORB vocabulary on the GPU (liborbfe.so): loading, and
 * TemplatedVocabulary::transform of a descriptor set into BowVector + FeatureVector.
 *
 * Replaces, for ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor, FORB>
 * (include/ORBVocabulary.h):
 *   loadFromTextFile    Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1351-1440  -> orbfe_vocab_load_text
 *   loadFromBinaryFile  TemplatedVocabulary.h:1467-1511                          -> orbfe_vocab_load_binary
 *   transform(features, BowVector&, FeatureVector&, levelsup)
 *                       TemplatedVocabulary.h:1140-1207 (+ per-descriptor descent :1231-1272,
 *                       BowVector::addWeight / addIfNotExist / normalize BowVector.cpp:35-85)
 *                                                        -> orbfe_vocab_transform(_batch_device)
 * called by Frame::ComputeBoW (Frame.cc:447-454) and KeyFrame::ComputeBoW (KeyFrame.cc:59-68)
 * with levelsup = 4. The FeatureVector feeds SearchByBoW / SearchForTriangulation, the BowVector
 * the KeyFrameDatabase scores.
 *
 * The tree is DBoW2's node table: node 0 is the root; every node i >= 1 names a parent and the
 * table must be a tree rooted at 0 (the files list parents before children); a node's
 * children are the nodes naming it as parent, in ascending id order (the loaders' push_back
 * order); a node with no children ends the descent; nodes flagged is_leaf get word ids 0,1,2..
 * in node order (the loaders' m_words); weights are WordValue = double.
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

/* DBoW2 enums (BowVector.h:29-53) */
enum { ORBFE_VOC_TF_IDF = 0, ORBFE_VOC_TF = 1, ORBFE_VOC_IDF = 2, ORBFE_VOC_BINARY = 3 };
enum {
  ORBFE_VOC_L1_NORM = 0, ORBFE_VOC_L2_NORM = 1, ORBFE_VOC_CHI_SQUARE = 2, ORBFE_VOC_KL = 3,
  ORBFE_VOC_BHATTACHARYYA = 4, ORBFE_VOC_DOT_PRODUCT = 5
};

typedef struct {
  int n_nodes;   /* including the root */
  int n_words;
  int k, levels; /* m_k, m_L */
  int scoring, weighting;
} orbfe_vocab_info;

/* From a node table (n_nodes >= 1; parent[0] is ignored). node_desc: n_nodes x 32 bytes.
 * device < 0 (here and in the loaders) keeps the table on the host only: get_info / export work,
 * transform returns ORBFE_ERR_STATE. */
int orbfe_vocab_create(int n_nodes, int k, int levels, int scoring, int weighting,
                       const int32_t* parent, const uint8_t* is_leaf, const uint8_t* node_desc,
                       const double* weights, int device, orbfe_vocabulary** out);
/* The reference's loaders. Text: header "k L scoring weighting", then one node per line
 * "parent is_leaf d0 .. d31 weight" (lines holding no token are skipped).
 * Binary: saveToBinaryFile's layout; like the reference, the final end-of-file iteration
 * appends a copy of the last node (never selected by the descent: same descriptor, later sibling). */
int orbfe_vocab_load_text(const char* path, int device, orbfe_vocabulary** out);
int orbfe_vocab_load_binary(const char* path, int device, orbfe_vocabulary** out);
int orbfe_vocab_get_info(const orbfe_vocabulary* v, orbfe_vocab_info* info);
/* Host copy of the node table (each pointer may be NULL; arrays sized n_nodes). word_id is the
 * Node::word_id the reference keeps (0 for nodes that are not words). */
int orbfe_vocab_export(const orbfe_vocabulary* v, int32_t* parent, uint8_t* is_leaf,
                       uint8_t* node_desc, double* weights, uint32_t* word_id);
int orbfe_vocab_destroy(orbfe_vocabulary* v);

/* transform of n descriptors (host memory), n <= 8192.
 * BowVector: bow_words[*n_words] ascending with bow_weights (may be NULL to skip);
 * FeatureVector as CSR: node_ids[*n_nodes], offsets[*n_nodes+1], indices[offsets[*n_nodes]]
 * (node ids ascending, features ascending inside a node). Buffers sized n (offsets n + 1). */
int orbfe_vocab_transform(orbfe_vocabulary* v, const uint8_t* desc, int n, int levelsup,
                          uint32_t* bow_words, double* bow_weights, int* n_words,
                          uint32_t* node_ids, int32_t* offsets, int32_t* indices, int* n_nodes);

/* Device batch: image i has d_counts[i] descriptors at d_desc + i*desc_stride. Its FeatureVector
 * goes to d_node_ids + i*cap, d_offsets + i*(cap+1), d_indices + i*cap, d_n_nodes[i]; its
 * BowVector to d_bow_words + i*cap, d_bow_weights + i*cap, d_bow_n[i] (all three NULL: the
 * FeatureVector only). cap <= 8192. The handle keeps its launch scratch per stream: batches
 * enqueued on different streams may run concurrently (the node table is read-only). */
int orbfe_vocab_transform_batch_device(orbfe_vocabulary* v, int n_images, const uint8_t* d_desc,
                                       size_t desc_stride, const int32_t* d_counts, int levelsup,
                                       uint32_t* d_bow_words, double* d_bow_weights,
                                       int32_t* d_bow_n, uint32_t* d_node_ids, int32_t* d_offsets,
                                       int32_t* d_indices, int32_t* d_n_nodes, int cap,
                                       void* stream);
#ifdef __cplusplus
}
#endif
#endif
