// iface_compat.h -- the index interfaces the JULEE/PMDFC server binds to,
// declared here so the facades build and are tested outside the reference
// tree.  Shapes (names, argument and return types) follow the reference's
// server/util/pair.h:6-11, server/IHash.h:9-22 and server/ICCEH.h:9-27.
// Inside the reference tree, define PMDFC_REFERENCE_HEADERS and put
// -I<reference>/server first: gpu_cceh.h then includes the real IHash.h and
// gpu_cceh_hybrid.h the real ICCEH.h (one of the two per translation unit:
// they share the include guard HASH_INTERFACE_H_).  Unlike the reference,
// this file declares both, so one test TU can drive both facades.
#pragma once
#ifndef PMDFC_IFACE_COMPAT_H_
#define PMDFC_IFACE_COMPAT_H_
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
#endif  // PMDFC_IFACE_COMPAT_H_
