// oracle/ref/sgsmooth_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// extern "C" binding of the reference's own CPSNWhere_SGSmooth
// (psn_where/PSNWhere_SGSmooth.{h,cpp}), compiled from the sources where they
// lie under /root/reference by oracle/Makefile (target _ref) into
// oracle/_ref/libsgsmooth_ref.so. Used only by tests/ to pin the SG smoother.
#include <deque>
#include <vector>

#include "PSNWhere_SGSmooth.h"

extern "C" {

void *sgref_create(int span, int degree) { return new CPSNWhere_SGSmooth(span, degree); }
void sgref_destroy(void *h) { delete static_cast<CPSNWhere_SGSmooth *>(h); }
// CPSNWhere_SGSmooth::Insert(double): returns refreshPos
int sgref_insert(void *h, double v) { return static_cast<CPSNWhere_SGSmooth *>(h)->Insert(v); }
int sgref_size(void *h) { return (int)static_cast<CPSNWhere_SGSmooth *>(h)->size(); }
double sgref_result(void *h, int pos) { return static_cast<CPSNWhere_SGSmooth *>(h)->GetResult(pos); }
// the Qset the reference computes (CalculateQ, static): Qbegin / Qmid / Qend
int sgref_q(int window, int degree, double *qbegin, double *qmid, double *qend) {
    Qset q = CPSNWhere_SGSmooth::CalculateQ(window, degree);
    for (size_t i = 0; i < q.Qbegin.size(); i++) qbegin[i] = q.Qbegin[i];
    for (size_t i = 0; i < q.Qmid.size(); i++) qmid[i] = q.Qmid[i];
    for (size_t i = 0; i < q.Qend.size(); i++) qend[i] = q.Qend[i];
    return (int)q.Qbegin.size();
}

}  // extern "C"
