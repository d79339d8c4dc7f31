/* A mock JNIEnv that runs jni/deltareplay_jni.c on the CPU without a JVM (tests/test_jni_glue.py):
 * objects are tagged heap cells, the JNI calls the glue makes are implemented from the JNI
 * specification, and every call made while an exception is pending (other than the calls the
 * specification allows then: ExceptionCheck, DeleteLocalRef, Release*) is counted as a violation.
 * The library side is a stub (tests/native/jni_stub_lib.c) whose answers each scenario sets.
 * Each scenario prints one line "name ok" or "name FAIL: why"; the exit status is the failure count. */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"
#include "deltareplay.h"

enum kind { K_CLASS, K_STRING, K_BYTES, K_LONGS, K_INTS, K_OBJS, K_BUF, K_THROW, K_METHOD };
struct _jobject {
  int kind;
  char name[128];     /* class name / method signature / throwable class */
  char* bytes;        /* string (UTF-8), byte array, throwable message */
  int64_t n;          /* array length / buffer capacity */
  int64_t* longs;
  int32_t* ints;
  jobject* objs;
  void* ptr;          /* direct buffer address */
};
struct _jmethodID {
  char cls[128], name[64], sig[128];
};

static jobject g_pending;       /* the pending exception */
static int g_violations;        /* JNI calls made while an exception was pending */
static int g_buffers;           /* NewDirectByteBuffer calls */
static int g_fail_buffer_at;    /* NewDirectByteBuffer call number that fails (0: none) */
static int g_array_reads;       /* Get<Type>ArrayElements / GetObjectArrayElement calls */

static void viol(void) {
  if (g_pending) ++g_violations;
}
static jobject mk(int kind) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  o->kind = kind;
  return o;
}
static jthrowable throwable(const char* cls, const char* msg) {
  jobject t = mk(K_THROW);
  snprintf(t->name, sizeof t->name, "%s", cls);
  t->bytes = strdup(msg ? msg : "");
  return t;
}

static jclass m_FindClass(JNIEnv* e, const char* name) {
  (void)e;
  viol();
  jobject c = mk(K_CLASS);
  snprintf(c->name, sizeof c->name, "%s", name);
  return c;
}
static jint m_Throw(JNIEnv* e, jthrowable t) { (void)e; viol(); g_pending = t; return 0; }
static jint m_ThrowNew(JNIEnv* e, jclass c, const char* msg) { (void)e; viol(); g_pending = throwable(c->name, msg); return 0; }
static jmethodID m_GetMethodID(JNIEnv* e, jclass c, const char* name, const char* sig) {
  (void)e;
  viol();
  struct _jmethodID* m = (struct _jmethodID*)calloc(1, sizeof *m);
  snprintf(m->cls, sizeof m->cls, "%s", c->name);
  snprintf(m->name, sizeof m->name, "%s", name);
  snprintf(m->sig, sizeof m->sig, "%s", sig);
  return m;
}
static jobject m_NewObject(JNIEnv* e, jclass c, jmethodID m, ...) {
  (void)e;
  viol();
  va_list ap;
  va_start(ap, m);
  jobject out = NULL;
  if (!strcmp(c->name, "java/lang/String") && !strcmp(m->sig, "([BLjava/lang/String;)V")) {
    jobject b = va_arg(ap, jobject), cs = va_arg(ap, jobject);
    if (strcmp(cs->bytes, "UTF-8")) { fprintf(stderr, "charset %s\n", cs->bytes); abort(); }
    out = mk(K_STRING);
    out->bytes = (char*)calloc((size_t)b->n + 1, 1);
    memcpy(out->bytes, b->bytes, (size_t)b->n);
    out->n = b->n;
  } else {  /* an exception class with a (String) / (Object) constructor */
    jobject s = va_arg(ap, jobject);
    out = throwable(c->name, s ? s->bytes : "");
  }
  va_end(ap);
  return out;
}
static jstring m_NewStringUTF(JNIEnv* e, const char* s) {
  (void)e;
  viol();
  jobject o = mk(K_STRING);
  o->bytes = strdup(s);
  o->n = (int64_t)strlen(s);
  return o;
}
static const char* m_GetStringUTFChars(JNIEnv* e, jstring s, jboolean* c) { (void)e; (void)c; viol(); return s->bytes; }
static void m_ReleaseStringUTFChars(JNIEnv* e, jstring s, const char* c) { (void)e; (void)s; (void)c; }
static jsize m_GetArrayLength(JNIEnv* e, jarray a) { (void)e; viol(); return (jsize)a->n; }
static jobjectArray m_NewObjectArray(JNIEnv* e, jsize n, jclass c, jobject init) {
  (void)e; (void)c; (void)init;
  viol();
  jobject a = mk(K_OBJS);
  a->n = n;
  a->objs = (jobject*)calloc((size_t)n + 1, sizeof(jobject));
  return a;
}
static jobject m_GetObjectArrayElement(JNIEnv* e, jobjectArray a, jsize i) {
  (void)e;
  viol();
  ++g_array_reads;
  if (i < 0 || i >= a->n) {
    g_pending = throwable("java/lang/ArrayIndexOutOfBoundsException", "");
    return NULL;
  }
  return a->objs[i];
}
static void m_SetObjectArrayElement(JNIEnv* e, jobjectArray a, jsize i, jobject v) {
  (void)e;
  viol();
  if (i < 0 || i >= a->n) { g_pending = throwable("java/lang/ArrayIndexOutOfBoundsException", ""); return; }
  a->objs[i] = v;
}
static jbyteArray m_NewByteArray(JNIEnv* e, jsize n) {
  (void)e;
  viol();
  jobject a = mk(K_BYTES);
  a->n = n;
  a->bytes = (char*)calloc((size_t)n + 1, 1);
  return a;
}
static jlongArray m_NewLongArray(JNIEnv* e, jsize n) {
  (void)e;
  viol();
  jobject a = mk(K_LONGS);
  a->n = n;
  a->longs = (int64_t*)calloc((size_t)n + 1, 8);
  return a;
}
static jbyte* m_GetByteArrayElements(JNIEnv* e, jbyteArray a, jboolean* c) { (void)e; (void)c; viol(); ++g_array_reads; return (jbyte*)a->bytes; }
static jint* m_GetIntArrayElements(JNIEnv* e, jintArray a, jboolean* c) { (void)e; (void)c; viol(); ++g_array_reads; return (jint*)a->ints; }
static jlong* m_GetLongArrayElements(JNIEnv* e, jlongArray a, jboolean* c) { (void)e; (void)c; viol(); ++g_array_reads; return (jlong*)a->longs; }
static void m_ReleaseByteArrayElements(JNIEnv* e, jbyteArray a, jbyte* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static void m_ReleaseIntArrayElements(JNIEnv* e, jintArray a, jint* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static void m_ReleaseLongArrayElements(JNIEnv* e, jlongArray a, jlong* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static void m_GetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, jbyte* out) {
  (void)e;
  viol();
  if (s < 0 || n < 0 || s + n > a->n) { g_pending = throwable("java/lang/ArrayIndexOutOfBoundsException", ""); return; }
  memcpy(out, a->bytes + s, (size_t)n);
}
static void m_SetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, const jbyte* in) {
  (void)e;
  viol();
  if (s < 0 || n < 0 || s + n > a->n) { g_pending = throwable("java/lang/ArrayIndexOutOfBoundsException", ""); return; }
  memcpy(a->bytes + s, in, (size_t)n);
}
static void m_SetLongArrayRegion(JNIEnv* e, jlongArray a, jsize s, jsize n, const jlong* in) {
  (void)e;
  viol();
  if (s < 0 || n < 0 || s + n > a->n) { g_pending = throwable("java/lang/ArrayIndexOutOfBoundsException", ""); return; }
  memcpy(a->longs + s, in, (size_t)n * 8);
}
static jobject m_NewDirectByteBuffer(JNIEnv* e, void* p, jlong cap) {
  (void)e;
  viol();
  ++g_buffers;
  if (cap > 0x7fffffffll || (g_fail_buffer_at && g_buffers == g_fail_buffer_at)) {
    g_pending = throwable("java/lang/IllegalArgumentException", "capacity");
    return NULL;
  }
  jobject b = mk(K_BUF);
  b->ptr = p;
  b->n = cap;
  return b;
}
static jboolean m_ExceptionCheck(JNIEnv* e) { (void)e; return g_pending != NULL; }
static void m_DeleteLocalRef(JNIEnv* e, jobject o) { (void)e; (void)o; }
static jint m_EnsureLocalCapacity(JNIEnv* e, jint n) { (void)e; (void)n; viol(); return 0; }

static const struct JNINativeInterface_ g_table = {
    m_FindClass, m_Throw, m_ThrowNew, m_GetMethodID, m_NewObject, m_NewStringUTF, m_GetStringUTFChars,
    m_ReleaseStringUTFChars, m_GetArrayLength, m_NewObjectArray, m_GetObjectArrayElement, m_SetObjectArrayElement,
    m_NewByteArray, m_NewLongArray, m_GetByteArrayElements, m_GetIntArrayElements, m_GetLongArrayElements,
    m_ReleaseByteArrayElements, m_ReleaseIntArrayElements, m_ReleaseLongArrayElements, m_GetByteArrayRegion,
    m_SetByteArrayRegion, m_SetLongArrayRegion, m_NewDirectByteBuffer, m_ExceptionCheck, m_DeleteLocalRef,
    m_EnsureLocalCapacity};
static JNIEnv g_envp = &g_table;
static JNIEnv* env = &g_envp;

/* ---- the stub library's knobs (tests/native/jni_stub_lib.c) ---- */
extern dr_export stub_export;
extern const char* stub_nonfile;
extern uint64_t stub_nonfile_len;
extern char stub_set_nonfile[256];
extern uint64_t stub_set_nonfile_len;
extern int stub_stage_calls;
extern const char* stub_error;

#define G(name) Java_org_apache_spark_sql_delta_gpu_DeltaReplayNative_00024_##name
jobjectArray G(export)(JNIEnv*, jobject, jlong, jint);
jobjectArray G(exportRange)(JNIEnv*, jobject, jlong, jint, jlong, jlong, jlongArray);
jlong G(stageNamedUtf8)(JNIEnv*, jobject, jlong, jbyteArray, jlongArray, jintArray, jintArray, jobjectArray, jobjectArray);
jbyteArray G(nonFileJsonUtf8)(JNIEnv*, jobject, jlong);
void G(setNonFileJsonUtf8)(JNIEnv*, jobject, jlong, jbyteArray, jboolean);
jlong G(replay)(JNIEnv*, jobject, jlong, jlong, jlong, jboolean);

static int g_fails;
static void reset(void) {
  g_pending = NULL;
  g_violations = g_buffers = g_fail_buffer_at = g_array_reads = 0;
}
static void report(const char* name, int ok, const char* why) {
  if (!ok || g_violations) {
    ++g_fails;
    printf("%s FAIL: %s (violations %d)\n", name, ok ? "JNI calls with an exception pending" : why, g_violations);
  } else {
    printf("%s ok\n", name);
  }
}
static jbyteArray bytes_of(const char* s, int64_t n) {
  jobject a = mk(K_BYTES);
  a->n = n;
  a->bytes = (char*)malloc((size_t)n + 1);
  memcpy(a->bytes, s, (size_t)n);
  return a;
}

static int64_t off3[3] = {0, 5, 9};
static int64_t offz[3] = {0, 0, 0};
static int64_t offbig[3] = {0, 5, 3000000000ll};
static uint8_t bytes9[16] = "abcdefghi";
static int64_t i2[2] = {1, 2};
static uint8_t u2[2] = {0, 1};

static void small_export(int64_t* path_off) {
  memset(&stub_export, 0, sizeof stub_export);
  stub_export.n = 2;
  stub_export.path_off = path_off; stub_export.path_bytes = bytes9;
  stub_export.size = i2; stub_export.modification_time = i2;
  stub_export.stats_off = off3; stub_export.stats_bytes = bytes9; stub_export.stats_null = u2;
  stub_export.pv_entry_off = offz; stub_export.pv_null = u2;
  stub_export.pv_key_off = offz; stub_export.pv_key_bytes = bytes9;
  stub_export.pv_val_off = offz; stub_export.pv_val_bytes = bytes9; stub_export.pv_val_null = u2;
  stub_export.tags_entry_off = offz; stub_export.tags_null = u2;
  stub_export.tags_key_off = offz; stub_export.tags_key_bytes = bytes9;
  stub_export.tags_val_off = offz; stub_export.tags_val_bytes = bytes9; stub_export.tags_val_null = u2;
}

int main(void) {
  /* 1. a side whose path bytes exceed a direct buffer: refused before any buffer */
  reset();
  small_export(offbig);
  jobjectArray r = G(export)(env, NULL, 1, 0);
  report("export_over_2gib_refused",
         !r && g_pending && !strcmp(g_pending->name, "java/lang/UnsupportedOperationException") && g_buffers == 0 &&
             strstr(g_pending->bytes, "exportRange") != NULL,
         "expected UnsupportedOperationException naming exportRange and no buffers");

  /* 2. a small side: 24 columns, exact capacities, null where the side has no column */
  reset();
  small_export(off3);
  r = G(export)(env, NULL, 1, 0);
  int ok = r && r->n == 24 && !g_pending && r->objs[0] && r->objs[0]->n == 24 && r->objs[1]->n == 9 &&
           r->objs[4] == NULL && r->objs[8]->n == 9;
  report("export_columns", ok, "expected 24 columns with exact capacities");

  /* 3. the JVM refuses the third buffer: the glue stops, no call while the exception is pending */
  reset();
  small_export(off3);
  g_fail_buffer_at = 3;
  r = G(export)(env, NULL, 1, 0);
  report("export_buffer_failure_stops", !r && g_pending && g_buffers == 3, "expected NULL after the failing buffer");

  /* 4. stage with a kinds array one short: IllegalArgumentException before any element is read */
  reset();
  jobject versions = mk(K_LONGS);
  versions->n = 2;
  versions->longs = i2;
  jobject kinds = mk(K_INTS);
  kinds->n = 1;
  kinds->ints = (int32_t*)calloc(1, 4);
  jobject parts = mk(K_INTS);
  parts->n = 2;
  parts->ints = (int32_t*)calloc(2, 4);
  jobject names = mk(K_OBJS);
  names->n = 2;
  names->objs = (jobject*)calloc(2, sizeof(jobject));
  jobject files = mk(K_OBJS);
  files->n = 2;
  files->objs = (jobject*)calloc(2, sizeof(jobject));
  const int before = stub_stage_calls;
  jlong h = G(stageNamedUtf8)(env, NULL, 1, bytes_of("/t/_delta_log", 13), versions, kinds, parts, names, files);
  report("stage_length_mismatch",
         h == 0 && g_pending && !strcmp(g_pending->name, "java/lang/IllegalArgumentException") && g_array_reads == 0 &&
             stub_stage_calls == before,
         "expected IllegalArgumentException with no element read and no stage call");

  /* 5. a null file byte array: IllegalArgumentException, the library is not called */
  reset();
  kinds->n = 2;
  kinds->ints = (int32_t*)calloc(2, 4);
  names->objs[0] = bytes_of("00000000000000000000.json", 25);
  names->objs[1] = bytes_of("00000000000000000001.json", 25);
  files->objs[0] = bytes_of("{}\n", 3);
  files->objs[1] = NULL;
  h = G(stageNamedUtf8)(env, NULL, 1, bytes_of("/t/_delta_log", 13), versions, kinds, parts, names, files);
  report("stage_null_element",
         h == 0 && g_pending && !strcmp(g_pending->name, "java/lang/IllegalArgumentException") &&
             stub_stage_calls == before,
         "expected IllegalArgumentException and no stage call");

  /* 6. UTF-8 text with a supplementary character (U+1D11E) crosses both ways unchanged */
  reset();
  static const char meta[] = "{\"metaData\":{\"description\":\"clef \xf0\x9d\x84\x9e\"}}";
  stub_nonfile = meta;
  stub_nonfile_len = sizeof meta - 1;
  jbyteArray out = G(nonFileJsonUtf8)(env, NULL, 1);
  ok = out && out->n == (int64_t)(sizeof meta - 1) && !memcmp(out->bytes, meta, sizeof meta - 1);
  G(setNonFileJsonUtf8)(env, NULL, 1, bytes_of(meta, sizeof meta - 1), 1);
  ok = ok && stub_set_nonfile_len == sizeof meta - 1 && !memcmp(stub_set_nonfile, meta, sizeof meta - 1);
  report("utf8_supplementary_roundtrip", ok && !g_pending, "bytes changed across the boundary");

  /* 7. an error message with a supplementary character becomes new String(bytes, "UTF-8") */
  reset();
  stub_error = "Versions of /t/\xf0\x9d\x84\x9e are not contiguous.";
  h = G(replay)(env, NULL, 1, 1, 0, 1);
  report("utf8_exception_message",
         h == 0 && g_pending && !strcmp(g_pending->name, "java/lang/IllegalStateException") &&
             !strcmp(g_pending->bytes, stub_error),
         "expected IllegalStateException with the exact UTF-8 message");

  /* 8. exportRange without a handle slot: IllegalArgumentException, the library is not called */
  reset();
  r = G(exportRange)(env, NULL, 1, 0, 0, 1, NULL);
  report("export_range_needs_handle", !r && g_pending && !strcmp(g_pending->name, "java/lang/IllegalArgumentException"),
         "expected IllegalArgumentException");

  /* 9. exportRange: the range's columns and its handle */
  reset();
  small_export(off3);
  jobject hs = mk(K_LONGS);
  hs->n = 1;
  hs->longs = (int64_t*)calloc(1, 8);
  r = G(exportRange)(env, NULL, 1, 0, 0, 2, hs);
  report("export_range_columns", r && r->n == 24 && hs->longs[0] != 0 && !g_pending, "expected columns and a handle");
  return g_fails;
}
