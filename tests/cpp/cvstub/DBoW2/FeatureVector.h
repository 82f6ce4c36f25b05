// TEST-ONLY stand-in for DBoW2's FeatureVector / BowVector (Thirdparty/DBoW2/DBoW2/FeatureVector.h,
// BowVector.h of the reference): std::maps keyed by node / word id, features in insertion order.
// The reference's headers reach every translation unit with `using namespace std` in scope
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:36, included through ORBVocabulary.h), and
// include/ORBmatcher.h relies on it (`vector<MapPoint*>`, `pair<size_t, size_t>`); so does this
// stub.
#ifndef ORBFE_TEST_STUB_DBOW2_FEATUREVECTOR_H
#define ORBFE_TEST_STUB_DBOW2_FEATUREVECTOR_H

#include <map>
#include <utility>
#include <vector>

namespace DBoW2 {
typedef unsigned int NodeId;
typedef unsigned int WordId;
typedef double WordValue;

class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {
 public:
  void addFeature(NodeId id, unsigned int i_feature) { (*this)[id].push_back(i_feature); }
};
class BowVector : public std::map<WordId, WordValue> {};
}  // namespace DBoW2

using namespace std;

#endif
