// edv_ledger.h -- ticket bookkeeping of the asynchronous host path
// (edv_verify_batch_async / edv_wait_async), plain C++ so the CPU test harness
// (libedv_hostcheck.so) checks the same code the library runs.
#pragma once
#include <stdint.h>

namespace edv {

// Tickets are issued in order.  A batch that fails marks the ledger: every
// later wait for a ticket at or below the highest failed one that no slot holds
// any more fails too.  Sticky, with no bounded list to fall out of, so a failed
// ticket can never be reported complete however many batches fail after it
// (fail closed: a batch that did complete before a later failure is reported
// failed as well).
struct AsyncLedger {
  int64_t next = 0;         // the next ticket to issue
  int64_t fail_floor = -1;  // highest failed ticket, -1 = none
  int64_t issue() { return next++; }
  void fail(int64_t t) {
    if (t > fail_floor) fail_floor = t;
  }
  // A wait for ticket t that no slot holds any more: 0 = complete, -1 (EDV_E_ARG)
  // = never issued, -3 (EDV_E_HIP) = failed.
  int settled(int64_t t) const {
    if (t < 0 || t >= next) return -1;
    return t <= fail_floor ? -3 : 0;
  }
  bool known(int64_t t) const { return t >= 0 && t < next; }
};

}  // namespace edv
