// ihash_compat.h -- the index interface the JULEE/PMDFC server binds to,
// declared here so the adapter builds and is tested outside the reference
// tree.  Shape (names, argument types, return types) follows the reference's
// server/IHash.h:9-22 and server/util/pair.h:6-11 exactly; inside the reference
// tree build with -DPMDFC_USE_REFERENCE_IHASH and -I<reference>/server so the
// real headers are used instead.
#pragma once
#if defined(PMDFC_USE_REFERENCE_IHASH)
#include "IHash.h"
#elif defined(PMDFC_USE_REFERENCE_ICCEH)
#include "ICCEH.h"  // shares IHash.h's include guard: one of the two per TU
#else
#include <cstddef>
#include <cstdint>
#include <vector>

typedef size_t Key_t;
typedef const char* Value_t;
const Key_t SENTINEL = -2;
const Key_t INVALID = -1;
const Value_t NONE = 0x0;

class IHash {
 public:
  IHash(void) = default;
  ~IHash(void) = default;
  virtual Key_t Insert(Key_t&, Value_t) = 0;
  virtual void Insert_extent(Key_t, uint64_t, uint64_t, Value_t) = 0;
  virtual bool Delete(Key_t&) = 0;
  virtual Value_t Get(Key_t&) = 0;
  virtual Value_t Get_extent(Key_t&, uint64_t) = 0;
  virtual Value_t FindAnyway(Key_t&) = 0;
  virtual double Utilization(void) = 0;
  virtual size_t Capacity(void) = 0;
  virtual bool Recovery(void) = 0;
};

// server/ICCEH.h:9-27 (CCEH_hybrid's flavour)
class ICCEH {
 public:
  ICCEH(void) = default;
  ~ICCEH(void) = default;
  virtual int GetNodeID(Key_t&) = 0;
  virtual void Insert_extent(Key_t, Value_t, uint64_t) = 0;
  virtual void Insert(Key_t&, Value_t) = 0;
  virtual bool Delete(Key_t&) = 0;
  virtual Value_t Get(Key_t&) = 0;
  virtual Value_t Get_extent(Key_t&) = 0;
  virtual Value_t FindAnyway(Key_t&) = 0;
  virtual double Utilization(void) = 0;
  virtual size_t Capacity(void) = 0;
  virtual bool Recovery(void) = 0;
  virtual std::vector<unsigned> Freqs(void) = 0;
  virtual std::vector<size_t> SegmentLoads(void) = 0;
  virtual std::vector<double> Metrics(void) = 0;
};
#endif
