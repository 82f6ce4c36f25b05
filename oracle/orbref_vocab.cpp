// orbref_vocab.cpp -- CPU oracle for the DBoW2 vocabulary (TEST INFRASTRUCTURE ONLY: loaded by
// tests/ and bench.py's parity legs as the checker, never by the product).
//
// Restates, for TemplatedVocabulary<FORB::TDescriptor, FORB> (Thirdparty/DBoW2/DBoW2/):
//   loadFromTextFile    TemplatedVocabulary.h:1351-1440 (stringstream extraction per line)
//   loadFromBinaryFile  TemplatedVocabulary.h:1467-1511 (fstream loop, eof tested before the read)
//   transform(features, BowVector&, FeatureVector&, levelsup)  :1140-1207, descent :1231-1272
//   BowVector::addWeight / addIfNotExist / normalize  BowVector.cpp:35-85
//   FeatureVector::addFeature  FeatureVector.cpp (std::map<NodeId, std::vector<unsigned>>)
// with the reference's containers (std::map, std::vector of child ids, double weights), so the
// GPU's sorted-key formulation is checked against the container semantics it replaces.
//
// Deterministic rules where the reference is undefined:
//   * a text line holding no token (the empty string getline returns after a final newline)
//     makes the reference extract an unset int parent; it is skipped here;
//   * when the descent ends above level m_L - levelsup, the reference leaves nid unset; the
//     final node stands in.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../include/orbfe.h"

namespace {

struct Node {  // TemplatedVocabulary::Node (TemplatedVocabulary.h:366-378)
  uint32_t id = 0;
  double weight = 0;
  std::vector<uint32_t> children;
  uint32_t parent = 0;
  uint8_t descriptor[32] = {};
  uint32_t word_id = 0;
  bool isLeaf() const { return children.empty(); }
};

int popcount_distance(const uint8_t* a, const uint8_t* b) {  // FORB::distance (FORB.cpp:61-80)
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

}  // namespace

struct orbref_vocab {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<Node> nodes;
  std::vector<uint32_t> words;  // m_words: node id of word w
};

extern "C" {

int orbref_vocab_load_text(const char* path, orbref_vocab** out) {
  std::ifstream f(path);
  if (!f.is_open() || !out) return ORBFE_ERR_ARG;
  auto* v = new orbref_vocab();
  std::string s;
  std::getline(f, s);
  std::stringstream ss;
  ss << s;
  int n1 = -1, n2 = -1;
  v->k = -1;
  v->L = -1;
  ss >> v->k >> v->L >> n1 >> n2;
  if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
    delete v;
    return ORBFE_ERR_ARG;
  }
  v->scoring = n1;
  v->weighting = n2;
  v->nodes.resize(1);
  v->nodes[0].id = 0;
  while (!f.eof()) {
    std::string snode;
    std::getline(f, snode);
    if (snode.find_first_not_of(" \t\r") == std::string::npos) continue;  // rule above
    std::stringstream ssnode;
    ssnode << snode;
    const uint32_t nid = (uint32_t)v->nodes.size();
    v->nodes.resize(v->nodes.size() + 1);
    v->nodes[nid].id = nid;
    int pid = -1;
    ssnode >> pid;
    if (pid < 0 || (uint32_t)pid >= nid) {
      delete v;
      return ORBFE_ERR_ARG;
    }
    v->nodes[nid].parent = (uint32_t)pid;
    v->nodes[pid].children.push_back(nid);
    int nIsLeaf = 0;
    ssnode >> nIsLeaf;
    std::stringstream ssd;  // FORB::fromString of the next 32 tokens
    for (int b = 0; b < 32; b++) {
      std::string e;
      ssnode >> e;
      ssd << e << " ";
    }
    for (int b = 0; b < 32; b++) {
      int x;
      ssd >> x;
      if (!ssd.fail()) v->nodes[nid].descriptor[b] = (unsigned char)x;
    }
    ssnode >> v->nodes[nid].weight;
    if (nIsLeaf > 0) {
      v->nodes[nid].word_id = (uint32_t)v->words.size();
      v->words.push_back(nid);
    }
  }
  *out = v;
  return ORBFE_OK;
}

int orbref_vocab_load_binary(const char* path, orbref_vocab** out) {
  std::fstream f;
  f.open(path, std::ios_base::in | std::ios::binary);
  if (!f.is_open() || !out) return ORBFE_ERR_ARG;
  unsigned int nb_nodes = 0, size_node = 0;
  auto* v = new orbref_vocab();
  f.read((char*)&nb_nodes, sizeof(nb_nodes));
  f.read((char*)&size_node, sizeof(size_node));
  f.read((char*)&v->k, sizeof(v->k));
  f.read((char*)&v->L, sizeof(v->L));
  f.read((char*)&v->scoring, sizeof(v->scoring));
  f.read((char*)&v->weighting, sizeof(v->weighting));
  if (!f || size_node < 41 || nb_nodes < 2) {
    delete v;
    return ORBFE_ERR_ARG;
  }
  v->nodes.resize(nb_nodes + 1);
  std::vector<char> buf(size_node, 0);
  uint32_t nid = 1;
  bool got_one = false;
  while (!f.eof()) {
    f.read(buf.data(), size_node);
    if (f.gcount() == (std::streamsize)size_node) got_one = true;
    else if (f.gcount() != 0) {  // a partial record: rejected (the library requires whole records)
      delete v;
      return ORBFE_ERR_ARG;
    }
    if (!got_one || nid >= v->nodes.size()) {  // would read an unfilled buffer / out of range
      delete v;
      return ORBFE_ERR_ARG;
    }
    Node& n = v->nodes[nid];
    n.id = nid;
    int32_t pid;
    memcpy(&pid, buf.data(), 4);
    if (pid < 0 || (uint32_t)pid >= v->nodes.size() || (uint32_t)pid == nid) {
      delete v;
      return ORBFE_ERR_ARG;
    }
    n.parent = (uint32_t)pid;
    v->nodes[pid].children.push_back(nid);
    memcpy(n.descriptor, buf.data() + 4, 32);
    float w;
    memcpy(&w, buf.data() + 36, 4);
    n.weight = w;
    if (buf[40]) {
      n.word_id = (uint32_t)v->words.size();
      v->words.push_back(nid);
    }
    nid++;
  }
  if (nid != v->nodes.size()) {  // the record count must be nb_nodes - 1 (+ the eof pass)
    delete v;
    return ORBFE_ERR_ARG;
  }
  *out = v;
  return ORBFE_OK;
}

int orbref_vocab_from_table(int n_nodes, int k, int levels, int scoring, int weighting,
                            const int32_t* parent, const uint8_t* is_leaf, const uint8_t* node_desc,
                            const double* weights, orbref_vocab** out) {
  if (n_nodes <= 0 || !out) return ORBFE_ERR_ARG;
  auto* v = new orbref_vocab();
  v->k = k;
  v->L = levels;
  v->scoring = scoring;
  v->weighting = weighting;
  v->nodes.resize(n_nodes);
  for (int i = 0; i < n_nodes; i++) {
    v->nodes[i].id = (uint32_t)i;
    memcpy(v->nodes[i].descriptor, node_desc + (size_t)i * 32, 32);
    v->nodes[i].weight = weights[i];
  }
  for (int i = 1; i < n_nodes; i++) {
    if (parent[i] < 0 || parent[i] >= n_nodes || parent[i] == i) {
      delete v;
      return ORBFE_ERR_ARG;
    }
    v->nodes[i].parent = (uint32_t)parent[i];
    v->nodes[parent[i]].children.push_back((uint32_t)i);
    if (is_leaf[i]) {
      v->nodes[i].word_id = (uint32_t)v->words.size();
      v->words.push_back((uint32_t)i);
    }
  }
  *out = v;
  return ORBFE_OK;
}

void orbref_vocab_free(orbref_vocab* v) { delete v; }

int orbref_vocab_info(const orbref_vocab* v, int* info6) {
  info6[0] = (int)v->nodes.size();
  info6[1] = (int)v->words.size();
  info6[2] = v->k;
  info6[3] = v->L;
  info6[4] = v->scoring;
  info6[5] = v->weighting;
  return ORBFE_OK;
}

int orbref_vocab_tables(const orbref_vocab* v, int32_t* parent, uint8_t* is_word, uint8_t* desc,
                        double* weight, uint32_t* word_id) {
  for (size_t i = 0; i < v->nodes.size(); i++) {
    parent[i] = i == 0 ? -1 : (int32_t)v->nodes[i].parent;
    memcpy(desc + i * 32, v->nodes[i].descriptor, 32);
    weight[i] = v->nodes[i].weight;
    word_id[i] = v->nodes[i].word_id;
    is_word[i] = 0;
  }
  for (uint32_t n : v->words) is_word[n] = 1;
  return ORBFE_OK;
}

// TemplatedVocabulary::transform (TemplatedVocabulary.h:1140-1207, 1231-1272)
int orbref_vocab_transform_full(const orbref_vocab* v, const uint8_t* desc, int n, int levelsup,
                                uint32_t* bow_words, double* bow_weights, int* n_words,
                                uint32_t* node_ids, int32_t* offsets, int32_t* indices,
                                int* n_nodes) {
  std::map<uint32_t, double> bow;                        // BowVector
  std::map<uint32_t, std::vector<unsigned>> fv;          // FeatureVector
  if (!v->words.empty()) {
    const bool must = v->scoring != 5;  // every scoring but DOT_PRODUCT normalises (ScoringObject.h:73-88)
    const int norm_l2 = v->scoring == 1;
    const bool additive = v->weighting == 0 || v->weighting == 1;  // TF_IDF, TF
    for (int i = 0; i < n; i++) {
      const uint8_t* feature = desc + (size_t)i * 32;
      const int nid_level = v->L - levelsup;
      uint32_t nid = 0;
      bool nid_set = nid_level <= 0;
      uint32_t final_id = 0;
      int current_level = 0;
      do {
        ++current_level;
        const std::vector<uint32_t>& nodes = v->nodes[final_id].children;
        final_id = nodes[0];
        double best_d = popcount_distance(feature, v->nodes[final_id].descriptor);
        for (size_t c = 1; c < nodes.size(); c++) {
          const double d = popcount_distance(feature, v->nodes[nodes[c]].descriptor);
          if (d < best_d) {
            best_d = d;
            final_id = nodes[c];
          }
        }
        if (current_level == nid_level) {
          nid = final_id;
          nid_set = true;
        }
      } while (!v->nodes[final_id].isLeaf());
      if (!nid_set) nid = final_id;  // rule above
      const uint32_t id = v->nodes[final_id].word_id;
      const double w = v->nodes[final_id].weight;
      if (w > 0) {
        if (additive) {  // BowVector::addWeight
          auto it = bow.lower_bound(id);
          if (it != bow.end() && !(id < it->first)) it->second += w;
          else bow.insert(it, {id, w});
        } else {  // BowVector::addIfNotExist
          auto it = bow.lower_bound(id);
          if (it == bow.end() || id < it->first) bow.insert(it, {id, w});
        }
        fv[nid].push_back((unsigned)i);  // FeatureVector::addFeature
      }
    }
    if (additive && !bow.empty() && !must) {
      const double nd = (double)bow.size();
      for (auto& e : bow) e.second /= nd;
    }
    if (must) {  // BowVector::normalize
      double norm = 0.0;
      if (!norm_l2) {
        for (auto& e : bow) norm += std::fabs(e.second);
      } else {
        for (auto& e : bow) norm += e.second * e.second;
        norm = std::sqrt(norm);
      }
      if (norm > 0.0)
        for (auto& e : bow) e.second /= norm;
    }
  }
  int w = 0;
  for (auto& e : bow) {
    if (bow_words) bow_words[w] = e.first;
    if (bow_weights) bow_weights[w] = e.second;
    w++;
  }
  if (n_words) *n_words = w;
  int k = 0, total = 0;
  for (auto& e : fv) {
    node_ids[k] = e.first;
    offsets[k] = total;
    for (unsigned f : e.second) indices[total++] = (int32_t)f;
    k++;
  }
  offsets[k] = total;
  *n_nodes = k;
  return ORBFE_OK;
}

}  // extern "C"
