/*!
 * \file dmlc/input_split_shuffle.h
 * \brief Coarse-grained shuffling: a rank's shard is cut into
 *  `num_shuffle_parts` sub-shards visited in a random order each epoch.
 * Parity: reference `include/dmlc/input_split_shuffle.h:19-166` (visiting
 * order from std::mt19937(666 + part + nparts + nshuffle + seed), reshuffled
 * on BeforeFirst, records chained across sub-shards).
 */
#ifndef DMLC_INPUT_SPLIT_SHUFFLE_H_
#define DMLC_INPUT_SPLIT_SHUFFLE_H_

#include <algorithm>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "./io.h"
#include "./logging.h"

namespace dmlc {

class InputSplitShuffle : public InputSplit {
 public:
  /*!
   * \param num_shuffle_parts sub-shards per rank (>1 to shuffle)
   * \param shuffle_seed seed of the visiting order
   */
  /*!
   * \brief the sub-shard visiting order of epoch `epoch` (0 = the order after
   *  construction, k = after k BeforeFirst calls) of a split created with the
   *  same arguments -- for readers that visit the sub-shards themselves (the
   *  GPU parser's shuffled mode)
   */
  static std::vector<unsigned> VisitOrder(unsigned part_index, unsigned num_parts,
                                          unsigned num_shuffle_parts, int shuffle_seed,
                                          unsigned epoch) {
    std::vector<unsigned> order(num_shuffle_parts);
    for (unsigned i = 0; i < num_shuffle_parts; ++i) order[i] = i;
    if (num_shuffle_parts <= 1) return order;
    std::mt19937 rnd(kRandMagic_ + part_index + num_parts + num_shuffle_parts + shuffle_seed);
    for (unsigned e = 0; e <= epoch; ++e) std::shuffle(order.begin(), order.end(), rnd);
    return order;
  }
  static InputSplit* Create(const char* uri, unsigned part_index, unsigned num_parts,
                            const char* type, unsigned num_shuffle_parts,
                            int shuffle_seed) {
    CHECK(num_shuffle_parts > 0) << "number of shuffle parts should be greater than zero!";
    if (num_shuffle_parts > 1) {
      return new InputSplitShuffle(uri, part_index, num_parts, type, num_shuffle_parts,
                                   shuffle_seed);
    }
    return InputSplit::Create(uri, part_index, num_parts, type);
  }

  InputSplitShuffle(const char* uri, unsigned part_index, unsigned num_parts,
                    const char* type, unsigned num_shuffle_parts, int shuffle_seed)
      : part_index_(part_index),
        num_parts_(num_parts),
        num_shuffle_parts_(num_shuffle_parts),
        cur_shuffle_idx_(0) {
    for (unsigned i = 0; i < num_shuffle_parts_; ++i) shuffle_indexes_.push_back(i);
    trnd_.seed(kRandMagic_ + part_index_ + num_parts_ + num_shuffle_parts_ + shuffle_seed);
    std::shuffle(shuffle_indexes_.begin(), shuffle_indexes_.end(), trnd_);
    source_.reset(InputSplit::Create(uri, SubPart(cur_shuffle_idx_), num_parts_ * num_shuffle_parts_,
                                     type));
  }
  void HintChunkSize(size_t chunk_size) override { source_->HintChunkSize(chunk_size); }
  size_t GetTotalSize() override { return source_->GetTotalSize(); }
  void BeforeFirst() override {
    if (num_shuffle_parts_ > 1) {
      std::shuffle(shuffle_indexes_.begin(), shuffle_indexes_.end(), trnd_);
      cur_shuffle_idx_ = 0;
      source_->ResetPartition(SubPart(cur_shuffle_idx_), num_parts_ * num_shuffle_parts_);
    } else {
      source_->BeforeFirst();
    }
  }
  /*!
   * \brief move to another rank's shard: the current visiting order is kept
   *  (no reshuffle), as in the reference (:75-80); part_index_ is updated so
   *  later sub-shards stay in the new shard (the reference keeps the old one).
   */
  void ResetPartition(unsigned part_index, unsigned num_parts) override {
    CHECK(num_parts == num_parts_) << "num_parts is not consistent!";
    CHECK(part_index < num_parts) << "invalid partition";
    part_index_ = part_index;
    cur_shuffle_idx_ = 0;
    source_->ResetPartition(SubPart(cur_shuffle_idx_), num_parts_ * num_shuffle_parts_);
  }
  bool NextRecord(Blob* out_rec) override {
    while (!source_->NextRecord(out_rec)) {
      if (!Advance()) return false;
    }
    return true;
  }
  bool NextChunk(Blob* out_chunk) override {
    while (!source_->NextChunk(out_chunk)) {
      if (!Advance()) return false;
    }
    return true;
  }

 private:
  static const int kRandMagic_ = 666;
  unsigned SubPart(unsigned idx) const {
    return part_index_ * num_shuffle_parts_ + shuffle_indexes_[idx];
  }
  bool Advance() {
    if (cur_shuffle_idx_ + 1 >= num_shuffle_parts_) return false;
    ++cur_shuffle_idx_;
    source_->ResetPartition(SubPart(cur_shuffle_idx_), num_parts_ * num_shuffle_parts_);
    return true;
  }
  unsigned part_index_;
  unsigned num_parts_;
  unsigned num_shuffle_parts_;
  unsigned cur_shuffle_idx_;
  std::vector<unsigned> shuffle_indexes_;
  std::mt19937 trnd_;
  std::unique_ptr<InputSplit> source_;
};
}  // namespace dmlc
#endif  // DMLC_INPUT_SPLIT_SHUFFLE_H_
