/* Stub libdeltareplay for tests/native/jni_mock.c: the entry points the mock scenarios reach return
 * what the scenario set; every other entry point the glue references is defined by
 * tests/test_jni_glue.py as a stub returning DR_E_INTERNAL (generated, no prototype needed). */
#include <string.h>

#include "deltareplay.h"

dr_export stub_export;
const char* stub_nonfile = "";
uint64_t stub_nonfile_len = 0;
char stub_set_nonfile[256];
uint64_t stub_set_nonfile_len = 0;
int stub_stage_calls = 0;
const char* stub_error = "";
static int stub_range;

int dr_state_export(dr_state* s, int32_t which, dr_export* out) {
  (void)s; (void)which;
  *out = stub_export;
  return DR_OK;
}
int dr_state_export_range(dr_state* s, int32_t which, int64_t lo, int64_t hi, dr_range** range, dr_export* out) {
  (void)s; (void)which; (void)lo; (void)hi;
  *out = stub_export;
  *range = (dr_range*)&stub_range;
  return DR_OK;
}
int dr_range_release(dr_range* r) { (void)r; return DR_OK; }
int dr_state_nonfile_json(dr_state* s, const char** json, uint64_t* len) {
  (void)s;
  *json = stub_nonfile;
  *len = stub_nonfile_len;
  return DR_OK;
}
int dr_state_set_nonfile_json(dr_state* s, const char* lines, uint64_t len, uint32_t flags) {
  (void)s; (void)flags;
  stub_set_nonfile_len = len < sizeof stub_set_nonfile ? len : sizeof stub_set_nonfile;
  memcpy(stub_set_nonfile, lines, (size_t)stub_set_nonfile_len);
  return DR_OK;
}
int dr_stage(dr_ctx* ctx, const dr_file* files, int32_t n, dr_staged** out) {
  (void)ctx; (void)files; (void)n; (void)out;
  ++stub_stage_calls;
  return DR_E_INTERNAL;
}
int dr_stage_named(dr_ctx* ctx, const char* lp, const dr_file* files, const char* const* names, int32_t n,
                   dr_staged** out) {
  (void)ctx; (void)lp; (void)files; (void)names; (void)n; (void)out;
  ++stub_stage_calls;
  return DR_E_INTERNAL;
}
int dr_replay_staged(dr_ctx* ctx, const dr_staged* st, int64_t cut, uint32_t flags, dr_state** out) {
  (void)ctx; (void)st; (void)cut; (void)flags; (void)out;
  return DR_E_NONCONTIGUOUS;
}
const char* dr_last_error(const dr_ctx* ctx) { (void)ctx; return stub_error; }
const char* dr_state_last_error(const dr_state* s) { (void)s; return stub_error; }
