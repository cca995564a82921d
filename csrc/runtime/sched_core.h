// Iteration-level (continuous-batching) scheduler core, pure C++17.
//
// The state machine behind runtime/scheduler.py. The Python `Scheduler`
// keeps the request futures, the sampling parameters and the GPU readout
// events; this core owns everything that changes at every decode step:
//   * sequences: slot, prefill progress, issued tokens, decode position,
//     sampler counter;
//   * per microbatch group: its decode rows, the sequences still
//     prefilling, and the composition of its last token-producing item;
//   * admission: a FIFO into free slots of the replica's SlotAllocator,
//     capped by the group capacity;
//   * planning: one step's group plans, i.e. leaves, joins, prefill chunks
//     under the token budget, decode rows, power-of-two row bucket and
//     256-position context bucket;
//   * readout assignment: sampled ids -> per-sequence events, EOS stop,
//     and slot release at a sequence's last item.
// The reference has no scheduler at all. Its coordinator runs one request's
// token loop per HTTP call (`server.py:154-206`); see SURVEY.md §5.2.
//
// Semantics are identical to the Python twin (`_PyCore` in
// runtime/scheduler.py); tests/test_sched_core.py drives both with the same
// random workloads and compares every plan and event.
#pragma once

#include <algorithm>
#include <cstdint>
#include <deque>
#include <map>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace lsd_rt {

// The free list the core allocates KV slots from (runtime.cpp binds the same
// class to Python as SlotAllocator).
class SlotAllocator {
 public:
  explicit SlotAllocator(int n) : cap_(n), used_(n, false) {
    for (int i = n - 1; i >= 0; --i) free_.push_back(i);
  }
  std::vector<int> alloc(int k) {
    if (k > (int)free_.size())
      throw std::runtime_error("out of KV slots: want " + std::to_string(k) + ", have " +
                               std::to_string(free_.size()));
    std::vector<int> out;
    out.reserve(k);
    for (int i = 0; i < k; ++i) {
      const int s = free_.back();
      free_.pop_back();
      used_[s] = true;
      out.push_back(s);
    }
    return out;
  }
  void free(const std::vector<int>& slots) {
    for (int s : slots) {
      if (s < 0 || s >= cap_ || !used_[s])
        throw std::runtime_error("double free / bad slot " + std::to_string(s));
      used_[s] = false;
      free_.push_back(s);
    }
  }
  int available() const { return (int)free_.size(); }
  int capacity() const { return cap_; }

 private:
  int cap_;
  std::vector<bool> used_;
  std::vector<int> free_;
};

// (sid, slot, start, len, final)
using ChunkOut = std::tuple<int64_t, int, int, int, bool>;
// (sid, slot, pos, sstep, src): src = index of the row's last token in the
// previous token-return vector of this group
using RowOut = std::tuple<int64_t, int, int, int, int>;
// (g, ret, n, b, ctxb, rows_changed, chunks, rows)
using GroupOut = std::tuple<int, int, int, int, int, bool, std::vector<ChunkOut>, std::vector<RowOut>>;
// (sid, token, flags): FIRST = first token of the sequence, FINISH = the
// request is complete now, RELEASE = its slot went back to the pool (token -1)
using Event = std::tuple<int64_t, int, int>;
constexpr int EV_FIRST = 1, EV_FINISH = 2, EV_RELEASE = 4;

class SchedCore {
 public:
  SchedCore(int replicas, int groups, int cap, int64_t prefill_budget, int chunk, int max_seq,
            std::vector<SlotAllocator*> pools)
      : R_(replicas), M_(groups), cap_(cap), budget_(prefill_budget), chunk_(chunk),
        max_seq_(max_seq), pools_(std::move(pools)),
        groups_(replicas, std::vector<Group>(groups)) {
    if ((int)pools_.size() != R_) throw std::invalid_argument("one slot pool per replica");
  }

  void add(int64_t sid, int prompt_len, int want, bool stop_at_eos) {
    if (prompt_len <= 0) throw std::invalid_argument("empty prompt");
    Seq s;
    s.prompt_len = prompt_len;
    s.want = want;
    s.stop_at_eos = stop_at_eos;
    seqs_[sid] = s;
    waiting_.push_back(sid);
  }

  // add() of a whole batch (one call from the scheduler's bulk admission)
  void add_many(const std::vector<int64_t>& sids, const std::vector<int>& prompt_lens,
                const std::vector<int>& wants, const std::vector<bool>& stops) {
    const size_t n = sids.size();
    if (prompt_lens.size() != n || wants.size() != n || stops.size() != n)
      throw std::invalid_argument("add_many: length mismatch");
    for (size_t i = 0; i < n; ++i)
      if (prompt_lens[i] <= 0) throw std::invalid_argument("empty prompt");
    for (size_t i = 0; i < n; ++i) add(sids[i], prompt_lens[i], wants[i], stops[i]);
  }

  bool has_work() const {
    if (!waiting_.empty()) return true;
    for (const auto& rep : groups_)
      for (const auto& g : rep)
        if (!g.rows.empty() || !g.prefilling.empty() || g.prev >= 0) return true;
    return false;
  }

  // Group plans of step `step` for every replica (groups with nothing to do
  // and nothing to read back are omitted); `admitted` gets the sequences
  // that joined at this step.
  std::vector<std::vector<GroupOut>> plan(int64_t step, std::vector<int64_t>* admitted) {
    std::vector<std::vector<GroupOut>> out(R_);
    for (int rep = 0; rep < R_; ++rep)
      for (int g = 0; g < M_; ++g) {
        GroupOut go;
        if (group_plan(rep, g, step, &go, admitted)) out[rep].push_back(std::move(go));
      }
    ++steps_;
    return out;
  }

  // Token readout of the item (rep, step, g): tokens = [decode rows | finals].
  std::vector<Event> assign(int rep, int64_t step, int g, const std::vector<int>& tokens, int eos) {
    auto it = expect_.find(key(rep, step, g));
    if (it == expect_.end()) throw std::runtime_error("no item awaiting this readout");
    const Produced prod = std::move(it->second);
    expect_.erase(it);
    std::vector<Event> ev;
    for (size_t i = 0; i < prod.rows.size(); ++i) give(prod.rows[i], tokens.at(i), eos, &ev);
    for (size_t j = 0; j < prod.finals.size(); ++j)
      give(prod.finals[j], tokens.at(prod.b + j), eos, &ev);
    for (int64_t sid : prod.release) release(sid, &ev);
    return ev;
  }

  // assign() for the serving hot path: each sequence's tokens are kept here,
  // and only FIRST / FINISH / RELEASE events come back (a plain token of a
  // running sequence costs the caller nothing), plus the whole token list of
  // every sequence that finished in this readout.  tokens points at n int32
  // ids (the pinned host copy of the token-return vector).
  using Finished = std::vector<std::pair<int64_t, std::vector<int>>>;
  std::pair<std::vector<Event>, Finished> assign_collect(int rep, int64_t step, int g,
                                                         const int32_t* tokens, int n, int eos) {
    auto it = expect_.find(key(rep, step, g));
    if (it == expect_.end()) throw std::runtime_error("no item awaiting this readout");
    const Produced prod = std::move(it->second);
    expect_.erase(it);
    auto tok_at = [&](size_t i) {
      if ((int)i >= n) throw std::out_of_range("token-return vector shorter than the item's rows");
      return (int)tokens[i];
    };
    std::vector<Event> ev;
    Finished done;
    for (size_t i = 0; i < prod.rows.size(); ++i) give_collect(prod.rows[i], tok_at(i), eos, &ev, &done);
    for (size_t j = 0; j < prod.finals.size(); ++j)
      give_collect(prod.finals[j], tok_at(prod.b + j), eos, &ev, &done);
    for (int64_t sid : prod.release) {
      auto f = seqs_.find(sid);
      if (f != seqs_.end() && !f->second.finished) done.emplace_back(sid, f->second.toks);
      release(sid, &ev);
    }
    return {std::move(ev), std::move(done)};
  }

  // Drop every sequence and give their slots back (failure path).
  void reset() {
    for (auto& kv : seqs_)
      if (kv.second.slot >= 0) pools_[kv.second.rep]->free({kv.second.slot});
    seqs_.clear();
    waiting_.clear();
    expect_.clear();
    produced_.clear();
    groups_.assign(R_, std::vector<Group>(M_));
  }

  // Join policy: a group admits waiting requests only when it has room for
  // all of them or for `join_min` of them, when it is idle, or after it has
  // deferred `max_wait` steps in a row -- so a running batch takes its
  // joiners in larger prefill items, fewer weight passes per generated token
  // (join_min 1: admit whatever fits at every step).
  void set_join_policy(int join_min, int max_wait) {
    if (join_min < 1 || max_wait < 0) throw std::invalid_argument("join_min >= 1, max_wait >= 0");
    join_min_ = join_min;
    max_wait_ = max_wait;
  }
  int64_t deferred() const { return deferred_; }

  int64_t joins() const { return joins_; }
  int64_t leaves() const { return leaves_; }
  int max_rows() const { return max_rows_; }
  int64_t steps() const { return steps_; }
  int n_waiting() const { return (int)waiting_.size(); }
  int n_seqs() const { return (int)seqs_.size(); }
  int n_expect() const { return (int)expect_.size(); }

 private:
  struct Seq {
    int rep = 0, g = -1, slot = -1;
    int prompt_len = 0, prefilled = 0, issued = 0, pos = 0, sstep = 1;
    int want = 0, ntok = 0;
    bool stop_at_eos = false, stop = false, finished = false;
    std::vector<int> toks;  // assign_collect only
  };
  struct Produced {
    int b = 0;
    std::vector<int64_t> rows, finals, release;
  };
  struct Group {
    std::vector<int64_t> rows, prefilling;
    // rows' Seq entries (node-based map: stable until a sequence is erased,
    // which happens only after it left its group), so the steady-state step
    // touches each row through a pointer instead of three hash lookups
    std::vector<Seq*> rowp;
    int64_t prev = -1;  // produced_ id of the last token-producing item
    int waited = 0;     // consecutive steps this group deferred its joins
  };

  static std::tuple<int, int64_t, int> key(int rep, int64_t step, int g) { return {rep, step, g}; }

  static int bucket(int n, int cap) {
    if (n <= 0) return 0;
    int b = 1;
    while (b < n) b <<= 1;
    return std::min(b, cap);
  }

  bool join_ok(Group& gh, int room, bool idle) {
    if (waiting_.empty() || room <= 0) {
      gh.waited = 0;
      return false;
    }
    if (idle || room >= std::min<int64_t>(join_min_, (int64_t)waiting_.size()) || gh.waited >= max_wait_) {
      gh.waited = 0;
      return true;
    }
    ++gh.waited;
    ++deferred_;
    return false;
  }

  std::vector<int64_t> admit(int rep, int g, int room, std::vector<int64_t>* admitted) {
    SlotAllocator* pool = pools_[rep];
    std::vector<int64_t> out;
    while (!waiting_.empty() && room > 0 && pool->available() > 0) {
      const int64_t sid = waiting_.front();
      waiting_.pop_front();
      Seq& s = seqs_.at(sid);
      s.rep = rep;
      s.g = g;
      s.slot = pool->alloc(1)[0];
      out.push_back(sid);
      if (admitted) admitted->push_back(sid);
      --room;
      ++joins_;
    }
    return out;
  }

  bool group_plan(int rep, int g, int64_t step, GroupOut* go, std::vector<int64_t>* admitted) {
    Group& gh = groups_[rep][g];
    int ret = 0, n = 0, b = 0, ctxb = 0;
    bool changed = false;
    std::vector<ChunkOut> chunks;
    std::vector<RowOut> rows;
    Produced* prev = nullptr;
    const int64_t prev_id = gh.prev;
    gh.prev = -1;
    if (prev_id >= 0) {
      prev = &produced_.at(prev_id);
      ret = prev->b + (int)prev->finals.size();
    }
    // leaves: every token scheduled, or EOS read back
    bool any_leave = false;
    for (const Seq* s : gh.rowp)
      if (s->issued >= s->want || s->stop) {
        any_leave = true;
        break;
      }
    // steady state (no leave, no newly sampled prefill): the rows stay put
    const bool same = !any_leave && !(prev && !prev->finals.empty());
    std::vector<int64_t> new_rows;
    std::vector<Seq*> new_p;
    if (same) {
      new_rows = gh.rows;
    } else {
      for (size_t i = 0; i < gh.rows.size(); ++i) {
        const int64_t sid = gh.rows[i];
        Seq* s = gh.rowp[i];
        if (s->issued >= s->want || s->stop) {
          ++leaves_;
          if (prev) prev->release.push_back(sid);
        } else {
          new_rows.push_back(sid);
          new_p.push_back(s);
        }
      }
      if (prev)
        for (int64_t sid : prev->finals) {
          new_rows.push_back(sid);
          new_p.push_back(&seqs_.at(sid));
        }
    }
    changed = !same && new_rows != gh.rows;
    // joins (capacity counts rows + sequences still prefilling)
    const int room = cap_ - (int)new_rows.size() - (int)gh.prefilling.size();
    if (join_ok(gh, room, new_rows.empty() && gh.prefilling.empty()))
      for (int64_t sid : admit(rep, g, room, admitted)) gh.prefilling.push_back(sid);
    // prefill chunks (FIFO, one chunk per sequence per step, token budget)
    int64_t budget = budget_ > 0 ? budget_ : (int64_t(1) << 62);
    std::vector<int64_t> finals;
    const std::vector<int64_t> pf = gh.prefilling;
    for (int64_t sid : pf) {
      Seq& s = seqs_.at(sid);
      const int L = s.prompt_len;
      const int take = chunk_ <= 0 ? L - s.prefilled : std::min(chunk_, L - s.prefilled);
      if (!chunks.empty() && take > budget) break;
      budget -= take;
      const int a = s.prefilled;
      const bool final = a + take == L;
      chunks.emplace_back(sid, s.slot, a, take, final);
      s.prefilled += take;
      if (final) {
        gh.prefilling.erase(std::find(gh.prefilling.begin(), gh.prefilling.end(), sid));
        finals.push_back(sid);
        s.issued = 1;
        s.pos = L;
        s.sstep = 1;
      }
    }
    // decode rows
    n = (int)new_rows.size();
    b = bucket(n, cap_);
    const std::vector<Seq*>& rp = same ? gh.rowp : new_p;
    if (changed) {
      std::unordered_map<int64_t, int> old_index;
      for (size_t i = 0; i < gh.rows.size(); ++i) old_index[gh.rows[i]] = (int)i;
      for (size_t k = 0; k < new_rows.size(); ++k) {
        const int64_t sid = new_rows[k];
        const Seq& s = *rp[k];
        int src;
        auto f = old_index.find(sid);
        if (f != old_index.end()) {
          src = f->second;
        } else {
          const auto p = std::find(prev->finals.begin(), prev->finals.end(), sid);
          src = prev->b + (int)(p - prev->finals.begin());
        }
        rows.emplace_back(sid, s.slot, s.pos, s.sstep, src);
      }
    }
    if (n) {
      int top = 0;
      for (const Seq* s : rp) top = std::max(top, s->pos);
      top += 1;
      ctxb = std::min((top + 255) / 256 * 256, max_seq_);
      for (Seq* s : rp) {  // one token per decode row this step
        s->issued += 1;
        s->pos += 1;
        s->sstep += 1;
      }
    }
    if (!same) {
      gh.rows = new_rows;
      gh.rowp = std::move(new_p);
    }
    max_rows_ = std::max(max_rows_, n);
    if (b || !finals.empty()) {
      Produced np;
      np.b = b;
      np.rows = new_rows;
      np.finals = finals;
      gh.prev = next_id_;
      produced_[next_id_++] = std::move(np);
    }
    if (prev) {  // its readout comes back in this step's token-return vector
      expect_[key(rep, step, g)] = std::move(*prev);
      produced_.erase(prev_id);
    }
    const bool has_work = b > 0 || !chunks.empty();
    if (!(ret || has_work)) return false;
    *go = GroupOut(g, ret, n, b, ctxb, changed, std::move(chunks), std::move(rows));
    return true;
  }

  void give(int64_t sid, int tok, int eos, std::vector<Event>* ev) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    Seq& s = it->second;
    if (s.finished || s.ntok >= s.want) return;
    int flags = s.ntok == 0 ? EV_FIRST : 0;
    s.ntok += 1;
    if (s.stop_at_eos && tok == eos) s.stop = true;
    if (s.ntok >= s.want || s.stop) {
      s.finished = true;
      flags |= EV_FINISH;
    }
    ev->emplace_back(sid, tok, flags);
  }

  void give_collect(int64_t sid, int tok, int eos, std::vector<Event>* ev, Finished* done) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    Seq& s = it->second;
    if (s.finished || s.ntok >= s.want) return;
    int flags = s.ntok == 0 ? EV_FIRST : 0;
    s.ntok += 1;
    s.toks.push_back(tok);
    if (s.stop_at_eos && tok == eos) s.stop = true;
    if (s.ntok >= s.want || s.stop) {
      s.finished = true;
      flags |= EV_FINISH;
      done->emplace_back(sid, s.toks);
    }
    if (flags) ev->emplace_back(sid, tok, flags);
  }

  void release(int64_t sid, std::vector<Event>* ev) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    const Seq s = it->second;
    seqs_.erase(it);
    if (s.slot >= 0) pools_[s.rep]->free({s.slot});
    ev->emplace_back(sid, -1, EV_RELEASE | (s.finished ? 0 : EV_FINISH));
  }

  int R_, M_, cap_;
  int64_t budget_;
  int chunk_, max_seq_;
  std::vector<SlotAllocator*> pools_;
  std::vector<std::vector<Group>> groups_;
  std::unordered_map<int64_t, Seq> seqs_;
  std::deque<int64_t> waiting_;
  std::map<std::tuple<int, int64_t, int>, Produced> expect_;
  std::unordered_map<int64_t, Produced> produced_;
  int64_t next_id_ = 0, joins_ = 0, leaves_ = 0, steps_ = 0, deferred_ = 0;
  int join_min_ = 1, max_wait_ = 0;
  int max_rows_ = 0;
};

}  // namespace lsd_rt
