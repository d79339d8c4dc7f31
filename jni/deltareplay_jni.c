/*
 * deltareplay_jni.c -- the JNI glue between the reference's Scala host and libdeltareplay.so.
 *
 * One native per method of `object DeltaReplayNative` (jni/DeltaReplayNative.scala, INTEGRATION.md
 * §1); Scala compiles an object's @native methods onto the module class `DeltaReplayNative$`, hence
 * the `_00024` in every symbol. Build (a maintainer, with the JDK's headers):
 *
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      jni/deltareplay_jni.c -Ldelta_amd -ldeltareplay -o libdeltareplay_jni.so
 *
 * Failures raise the reference's exception classes with the library's message (the reference's own
 * texts, D/DeltaErrors.scala:451-560, D/Snapshot.scala:334-345) -- see throw_status. Handles cross
 * the boundary as jlong; the Scala side owns their lifetime (release / stagedRelease / ctxDestroy /
 * rangeRelease). Export columns are wrapped zero-copy with NewDirectByteBuffer: they stay valid until
 * the state (export) or the range (exportRange) is released, which is the lifetime Snapshot.uncache
 * gives the cached state (D/util/StateCache.scala:104-109). A direct buffer holds at most 2^31 - 1
 * bytes: export refuses a side with a larger column (UnsupportedOperationException) and the host
 * takes it as row ranges (exportPlan / exportRange, ABI 3) instead.
 *
 * Text crosses as UTF-8 byte arrays in both directions (the *Utf8 natives; Scala converts with
 * StandardCharsets.UTF_8): JNI's own string calls speak modified UTF-8, which encodes characters
 * outside the BMP as surrogate pairs and U+0000 as C0 80, so table paths or metaData values with such
 * characters would not survive them. Exception messages are built as new String(bytes, "UTF-8") too.
 * No JNI call is made while an exception is pending: every call that can raise one is checked.
 *
 * Paths: D/ = core/src/main/scala/org/apache/spark/sql/delta/.
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "deltareplay.h"

#define NATIVE(ret, name) JNIEXPORT ret JNICALL Java_org_apache_spark_sql_delta_gpu_DeltaReplayNative_00024_##name

/* ---- errors and strings --------------------------------------------------------------------------- */

static int pending(JNIEnv* env) { return (*env)->ExceptionCheck(env) ? 1 : 0; }

/* new String(bytes[0..n), "UTF-8"): the library's standard UTF-8 as a Java string (NULL with an
 * exception pending on failure). */
static jstring utf8_string(JNIEnv* env, const char* bytes, size_t n) {
  if (n > 0x7fffffffu) n = 0x7fffffffu;
  jbyteArray b = (*env)->NewByteArray(env, (jsize)n);
  if (!b) return NULL;
  if (n) (*env)->SetByteArrayRegion(env, b, 0, (jsize)n, (const jbyte*)bytes);
  jclass sc = (*env)->FindClass(env, "java/lang/String");
  jmethodID ctor = sc ? (*env)->GetMethodID(env, sc, "<init>", "([BLjava/lang/String;)V") : NULL;
  jstring cs = ctor ? (*env)->NewStringUTF(env, "UTF-8") : NULL;  /* ASCII: modified UTF-8 is UTF-8 */
  jstring out = cs ? (jstring)(*env)->NewObject(env, sc, ctor, b, cs) : NULL;
  (*env)->DeleteLocalRef(env, b);
  if (sc) (*env)->DeleteLocalRef(env, sc);
  if (cs) (*env)->DeleteLocalRef(env, cs);
  return out;
}

/* bytes[0..n) as a new byte[] (NULL with an exception pending on failure). */
static jbyteArray byte_array(JNIEnv* env, const void* bytes, uint64_t n) {
  if (n > 0x7fffffffull) {
    jclass c = (*env)->FindClass(env, "java/lang/UnsupportedOperationException");
    if (c) (*env)->ThrowNew(env, c, "result over 2 GiB");
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, (jsize)n);
  if (out && n) (*env)->SetByteArrayRegion(env, out, 0, (jsize)n, (const jbyte*)bytes);
  return out;
}

/* The reference's exception for a dr_status (error mapping), with the library's UTF-8
 * message. AssertionError has no (String) constructor, so it is built through its (Object) one.
 * DR_E_REBUILD is not an error: the callers that can see it return 0 and the Scala side rebuilds the
 * snapshot from its segment. */
static void throw_status(JNIEnv* env, int rc, const char* msg) {
  const char* cls;
  const char* sig = "(Ljava/lang/String;)V";
  switch (rc) {
    case DR_E_EMPTY_DIR:
    case DR_E_LOG_TRUNCATED:
    case DR_E_IO: cls = "java/io/FileNotFoundException"; break;
    case DR_E_MISSING_PART:
    case DR_E_NONCONTIGUOUS:
    case DR_E_MISSING_PROTOCOL:
    case DR_E_MISSING_METADATA:
    case DR_E_CHECKSUM:
    case DR_E_INTERNAL: cls = "java/lang/IllegalStateException"; break;
    case DR_E_BAD_SEGMENT:
    case DR_E_INVALID_ARG: cls = "java/lang/IllegalArgumentException"; break;
    case DR_E_UNSUPPORTED: cls = "java/lang/UnsupportedOperationException"; break;
    case DR_E_OOM: cls = "java/lang/OutOfMemoryError"; break;
    case DR_E_FOREIGN_FILE: cls = "java/lang/AssertionError"; sig = "(Ljava/lang/Object;)V"; break;
    default: cls = "java/lang/RuntimeException"; break; /* DR_E_PARSE, DR_E_PARQUET, DR_E_DEVICE, ... */
  }
  if (pending(env)) return;
  if (!msg || !*msg) msg = "libdeltareplay call failed";
  jclass c = (*env)->FindClass(env, cls);
  jmethodID ctor = c ? (*env)->GetMethodID(env, c, "<init>", sig) : NULL;
  jstring s = ctor ? utf8_string(env, msg, strlen(msg)) : NULL;
  jobject ex = s ? (*env)->NewObject(env, c, ctor, s) : NULL;
  if (ex) (*env)->Throw(env, (jthrowable)ex);
}

#define CHECK_CTX(env, rc, ctx, ret)                                   \
  do {                                                                 \
    if ((rc) != DR_OK) {                                               \
      throw_status(env, rc, dr_last_error((const dr_ctx*)(ctx)));      \
      return ret;                                                      \
    }                                                                  \
  } while (0)
#define CHECK_STATE(env, rc, st, ret)                                  \
  do {                                                                 \
    if ((rc) != DR_OK) {                                               \
      throw_status(env, rc, dr_state_last_error((const dr_state*)(st))); \
      return ret;                                                      \
    }                                                                  \
  } while (0)

static jlongArray long_array(JNIEnv* env, const int64_t* v, int64_t n) {
  if (n < 0 || n > 0x7fffffff) {
    throw_status(env, DR_E_UNSUPPORTED, "result over 2^31 - 1 elements");
    return NULL;
  }
  jlongArray out = (*env)->NewLongArray(env, (jsize)n);
  if (out && n) (*env)->SetLongArrayRegion(env, out, 0, (jsize)n, (const jlong*)v);
  return out;
}

/* A UTF-8 byte[] (String.getBytes(UTF_8) on the Scala side) as a NUL-terminated copy the caller
 * frees; NULL for a null array or on failure. */
static char* utf8_copy(JNIEnv* env, jbyteArray b) {
  if (!b) return NULL;
  const jsize n = (*env)->GetArrayLength(env, b);
  char* out = (char*)malloc((size_t)n + 1);
  if (!out) return NULL;
  if (n) (*env)->GetByteArrayRegion(env, b, 0, n, (jbyte*)out);
  out[n] = 0;
  if (pending(env)) {
    free(out);
    return NULL;
  }
  return out;
}

/* ---- context ----------------------------------------------------------------------------------- */

NATIVE(jint, abiVersion)(JNIEnv* env, jobject self) {
  (void)env; (void)self;
  return dr_abi_version();   /* the Scala side refuses a library whose version != DR_ABI_VERSION */
}

NATIVE(jlong, ctxCreate)(JNIEnv* env, jobject self, jint device) {
  (void)self;
  dr_ctx* ctx = NULL;
  int rc = dr_ctx_create(device, &ctx);
  if (rc != DR_OK) {
    throw_status(env, rc, "dr_ctx_create: no usable HIP device");
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

NATIVE(void, ctxDestroy)(JNIEnv* env, jobject self, jlong ctx) {
  (void)env; (void)self;
  dr_ctx_destroy((dr_ctx*)(intptr_t)ctx);
}

/* dr_ctx_set_option (ABI 4): the session's configuration of the path (DeltaSQLConf); a rejected
 * option or value raises IllegalArgumentException with the library's message. */
NATIVE(void, setOption)(JNIEnv* env, jobject self, jlong ctx, jint option, jlong value) {
  (void)self;
  if (dr_ctx_set_option((dr_ctx*)(intptr_t)ctx, (int32_t)option, (int64_t)value) != DR_OK) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (c) (*env)->ThrowNew(env, c, "dr_ctx_set_option: option or value not accepted");
  }
}

NATIVE(jbyteArray, lastErrorUtf8)(JNIEnv* env, jobject self, jlong ctx) {
  (void)self;
  const char* m = dr_last_error((const dr_ctx*)(intptr_t)ctx);
  return byte_array(env, m ? m : "", m ? strlen(m) : 0);
}

/* ---- staging ----------------------------------------------------------------------------------- */

/* Snapshot.stateReconstruction's input (D/Snapshot.scala:88-111): the LogSegment of `version`
 * (< 0: latest) listed and read by the library (SnapshotManagement.getLogSegmentForVersion). */
NATIVE(jlong, stageLogUtf8)(JNIEnv* env, jobject self, jlong ctx, jbyteArray log_path, jlong version) {
  (void)self;
  char* path = utf8_copy(env, log_path);
  if (pending(env)) return 0;
  dr_staged* st = NULL;
  int rc = path ? dr_stage_log((dr_ctx*)(intptr_t)ctx, path, (int64_t)version, &st) : DR_E_INVALID_ARG;
  free(path);
  CHECK_CTX(env, rc, (intptr_t)ctx, 0);
  return (jlong)(intptr_t)st;
}

/* One rank's slice of the segment for the sharded replay (dr_shard_plan's cut). */
NATIVE(jlong, stageLogShardUtf8)(JNIEnv* env, jobject self, jlong ctx, jbyteArray log_path, jlong version,
                                 jint world, jint rank) {
  (void)self;
  char* path = utf8_copy(env, log_path);
  if (pending(env)) return 0;
  dr_staged* st = NULL;
  int rc = path ? dr_stage_log_shard((dr_ctx*)(intptr_t)ctx, path, (int64_t)version, world, rank, &st)
                : DR_E_INVALID_ARG;
  free(path);
  CHECK_CTX(env, rc, (intptr_t)ctx, 0);
  return (jlong)(intptr_t)st;
}

/* Files the host read itself. kinds[i] (dr_file_kind), parts[i] (1-based checkpoint part, 0 for a
 * commit or a single-part checkpoint); with `log_path` and `names` (UTF-8 byte arrays) non-null every
 * file is checked to belong to the table (assertLogBelongsToTable, D/Snapshot.scala:102,334-345).
 * Every parallel array must hold one entry per version (IllegalArgumentException otherwise, before
 * any element is read). The file bytes are copied into HBM during the call, so the Java arrays are
 * released before it returns; the byte arrays stay pinned together for the call, so the local
 * reference capacity is raised to hold them. */
static jlong stage_files(JNIEnv* env, jlong ctx, jbyteArray log_path, jlongArray versions, jintArray kinds,
                         jintArray parts, jobjectArray names, jobjectArray bytes) {
  const jsize n = versions ? (*env)->GetArrayLength(env, versions) : 0;
  if (!bytes || (*env)->GetArrayLength(env, bytes) != n || (kinds && (*env)->GetArrayLength(env, kinds) != n) ||
      (parts && (*env)->GetArrayLength(env, parts) != n) || (names && (*env)->GetArrayLength(env, names) != n)) {
    throw_status(env, DR_E_INVALID_ARG, "stage: versions, kinds, parts, names and bytes must have equal lengths");
    return 0;
  }
  if (n > 0 && (*env)->EnsureLocalCapacity(env, n + 16) != 0) return 0;  /* OutOfMemoryError pending */
  dr_file* files = (dr_file*)calloc((size_t)n + 1, sizeof(dr_file));
  jbyteArray* arrs = (jbyteArray*)calloc((size_t)n + 1, sizeof(jbyteArray));
  jbyte** data = (jbyte**)calloc((size_t)n + 1, sizeof(jbyte*));
  char** cnames = (char**)calloc((size_t)n + 1, sizeof(char*));
  jlong* v = n ? (*env)->GetLongArrayElements(env, versions, NULL) : NULL;
  jint* k = (n && kinds) ? (*env)->GetIntArrayElements(env, kinds, NULL) : NULL;
  jint* p = (n && parts) ? (*env)->GetIntArrayElements(env, parts, NULL) : NULL;
  int rc = DR_OK;
  if (!files || !arrs || !data || !cnames || (n && (!v || (kinds && !k) || (parts && !p)))) rc = DR_E_OOM;
  for (jsize i = 0; i < n && rc == DR_OK; ++i) {
    arrs[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, bytes, i);
    data[i] = arrs[i] ? (*env)->GetByteArrayElements(env, arrs[i], NULL) : NULL;
    if (!data[i]) { rc = -1; break; }
    files[i].version = (int64_t)v[i];
    files[i].kind = k ? k[i] : DR_FILE_JSON;
    files[i].part = p ? p[i] : 0;
    files[i].data = (const uint8_t*)data[i];
    files[i].len = (uint64_t)(*env)->GetArrayLength(env, arrs[i]);
    if (names) {
      jbyteArray nm = (jbyteArray)(*env)->GetObjectArrayElement(env, names, i);
      cnames[i] = utf8_copy(env, nm);
      if (nm) (*env)->DeleteLocalRef(env, nm);
      if (!cnames[i]) { rc = -1; break; }
    }
  }
  dr_staged* st = NULL;
  char* path = log_path ? utf8_copy(env, log_path) : NULL;
  if (rc == DR_OK && pending(env)) rc = -1;
  if (rc == DR_OK) {
    rc = names ? dr_stage_named((dr_ctx*)(intptr_t)ctx, path ? path : "", files, (const char* const*)cnames, n, &st)
               : dr_stage((dr_ctx*)(intptr_t)ctx, files, n, &st);
  }
  for (jsize i = 0; i < n && arrs; ++i) {
    if (data && data[i]) (*env)->ReleaseByteArrayElements(env, arrs[i], data[i], JNI_ABORT);
    if (arrs[i]) (*env)->DeleteLocalRef(env, arrs[i]);
    if (cnames) free(cnames[i]);
  }
  if (v) (*env)->ReleaseLongArrayElements(env, versions, v, JNI_ABORT);
  if (k) (*env)->ReleaseIntArrayElements(env, kinds, k, JNI_ABORT);
  if (p) (*env)->ReleaseIntArrayElements(env, parts, p, JNI_ABORT);
  free(path); free(files); free(arrs); free(data); free(cnames);
  if (pending(env)) return 0;  /* e.g. a null element: NullPointerException / ArrayIndexOutOfBounds */
  if (rc == DR_E_OOM) {
    throw_status(env, rc, "stage: out of host memory");
    return 0;
  }
  if (rc == -1) {
    throw_status(env, DR_E_INVALID_ARG, "stage: a null byte array or name");
    return 0;
  }
  CHECK_CTX(env, rc, (intptr_t)ctx, 0);
  return (jlong)(intptr_t)st;
}

/* Commit files after snapshot.version, for `apply` (SnapshotManagement.update). */
NATIVE(jlong, stage)(JNIEnv* env, jobject self, jlong ctx, jlongArray versions, jobjectArray bytes) {
  (void)self;
  return stage_files(env, ctx, NULL, versions, NULL, NULL, NULL, bytes);
}

NATIVE(jlong, stageNamedUtf8)(JNIEnv* env, jobject self, jlong ctx, jbyteArray log_path, jlongArray versions,
                              jintArray kinds, jintArray parts, jobjectArray names, jobjectArray bytes) {
  (void)self;
  return stage_files(env, ctx, log_path, versions, kinds, parts, names, bytes);
}

NATIVE(void, stagedRelease)(JNIEnv* env, jobject self, jlong staged) {
  (void)env; (void)self;
  dr_staged_release((dr_staged*)(intptr_t)staged);
}

/* ---- replay ------------------------------------------------------------------------------------ */

/* Snapshot.stateReconstruction + computedState (D/Snapshot.scala:88-176); validate =
 * DELTA_STATE_RECONSTRUCTION_VALIDATION_ENABLED (D/sources/DeltaSQLConf.scala:86-91). */
NATIVE(jlong, replay)(JNIEnv* env, jobject self, jlong ctx, jlong staged, jlong min_file_retention_ts,
                      jboolean validate) {
  (void)self;
  dr_state* st = NULL;
  int rc = dr_replay_staged((dr_ctx*)(intptr_t)ctx, (const dr_staged*)(intptr_t)staged,
                            (int64_t)min_file_retention_ts, validate ? 0u : DR_FLAG_NO_VALIDATION, &st);
  CHECK_CTX(env, rc, (intptr_t)ctx, 0);
  return (jlong)(intptr_t)st;
}

/* SnapshotManagement.update (D/SnapshotManagement.scala:286-330) as an O(tail) extension of `state`;
 * 0 without an exception = DR_E_REBUILD (replay the new segment instead). */
NATIVE(jlong, apply)(JNIEnv* env, jobject self, jlong ctx, jlong state, jlong tail, jlong min_file_retention_ts,
                     jboolean validate) {
  (void)self;
  dr_state* st = NULL;
  int rc = dr_state_apply((dr_ctx*)(intptr_t)ctx, (dr_state*)(intptr_t)state, (const dr_staged*)(intptr_t)tail,
                          (int64_t)min_file_retention_ts, validate ? 0u : DR_FLAG_NO_VALIDATION, &st);
  if (rc == DR_E_REBUILD) return 0;
  CHECK_CTX(env, rc, (intptr_t)ctx, 0);
  return (jlong)(intptr_t)st;
}

NATIVE(void, release)(JNIEnv* env, jobject self, jlong state) {
  (void)env; (void)self;
  dr_state_release((dr_state*)(intptr_t)state);
}

static jlongArray counts_array(JNIEnv* env, const dr_counts* c) {
  /* the order of DeltaReplayNative.CountFields */
  const int64_t v[12] = {c->num_files, c->size_in_bytes, c->num_removes, c->num_metadata, c->num_protocol,
                         c->num_set_transactions, c->num_actions, c->num_file_actions, c->version,
                         c->malformed_lines, (int64_t)c->live_key_sum, (int64_t)c->tomb_key_sum};
  return long_array(env, v, 12);
}

/* computedState (D/Snapshot.scala:136-176): numOfFiles, sizeInBytes, numOfRemoves, numOfMetadata,
 * numOfProtocol, setTransactions.size, then the replay's own figures. */
NATIVE(jlongArray, counts)(JNIEnv* env, jobject self, jlong state) {
  (void)self;
  dr_counts c;
  int rc = dr_state_counts((dr_state*)(intptr_t)state, &c);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  return counts_array(env, &c);
}

NATIVE(jlongArray, localCounts)(JNIEnv* env, jobject self, jlong state) {
  (void)self;
  dr_counts c;
  int rc = dr_state_local_counts((dr_state*)(intptr_t)state, &c);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  return counts_array(env, &c);
}

/* Latest protocol / metaData and the set transactions, one {"protocol":...} / {"metaData":...} /
 * {"txn":...} line each: the Scala side decodes them with Action.fromJson (D/actions/actions.scala:57-59). */
NATIVE(jbyteArray, nonFileJsonUtf8)(JNIEnv* env, jobject self, jlong state) {
  (void)self;
  const char* json = NULL;
  uint64_t len = 0;
  int rc = dr_state_nonfile_json((dr_state*)(intptr_t)state, &json, &len);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  return byte_array(env, json, len);
}

/* A sharded state's table-wide non-file winners when the host drove the exchange itself. */
NATIVE(void, setNonFileJsonUtf8)(JNIEnv* env, jobject self, jlong state, jbyteArray lines, jboolean validate) {
  (void)self;
  const jsize n = lines ? (*env)->GetArrayLength(env, lines) : 0;
  char* z = utf8_copy(env, lines);
  if (pending(env)) return;
  int rc = dr_state_set_nonfile_json((dr_state*)(intptr_t)state, z ? z : "", z ? (uint64_t)n : 0,
                                     validate ? 0u : DR_FLAG_NO_VALIDATION);
  free(z);
  CHECK_STATE(env, rc, (intptr_t)state, );
}

/* ValidateChecksum (D/Checksum.scala:155-191): null when the counters match or the .crc is absent or
 * unreadable (checksumOpt = None), else checkMismatch's text for the caller's IllegalStateException. */
NATIVE(jbyteArray, checkChecksumUtf8)(JNIEnv* env, jobject self, jlong state, jbyteArray crc_line) {
  (void)self;
  const jsize n = crc_line ? (*env)->GetArrayLength(env, crc_line) : 0;
  jbyte* b = crc_line ? (*env)->GetByteArrayElements(env, crc_line, NULL) : NULL;
  char msg[4096];
  uint64_t mlen = 0;
  int rc = dr_state_check_checksum((dr_state*)(intptr_t)state, (const char*)b, (uint64_t)n, msg, sizeof msg, &mlen);
  if (b) (*env)->ReleaseByteArrayElements(env, crc_line, b, JNI_ABORT);
  if (rc == DR_OK || rc == DR_E_NO_CHECKSUM) return NULL;
  if (rc != DR_E_CHECKSUM) {
    throw_status(env, rc, dr_state_last_error((const dr_state*)(intptr_t)state));
    return NULL;
  }
  return byte_array(env, msg, strlen(msg));
}

/* Order-free full-record checksums (parity gate): {live, tombstones}. */
NATIVE(jlongArray, recordSums)(JNIEnv* env, jobject self, jlong state) {
  (void)self;
  uint64_t l = 0, t = 0;
  int rc = dr_state_record_sums((dr_state*)(intptr_t)state, &l, &t);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  const int64_t v[2] = {(int64_t)l, (int64_t)t};
  return long_array(env, v, 2);
}

/* ---- allFiles / tombstones as SingleAction columns ---------------------------------------------- */

/* A direct ByteBuffer over p[0..bytes); `*failed` is set when the JVM raised (the caller stops). */
static jobject direct(JNIEnv* env, const void* p, int64_t bytes, int* failed) {
  if (*failed || !p) return NULL;
  /* a zero-length column still gets a buffer (an empty table has n + 1 = 1 offsets) */
  jobject b = (*env)->NewDirectByteBuffer(env, (void*)p, (jlong)bytes);
  if (!b || pending(env)) *failed = 1;
  return b;
}

#define DR_EXPORT_COLS 24
/* The byte size of every dr_export column, in declaration order (DeltaReplayNative.ExportColumns). */
static void column_sizes(const dr_export* e, const void* ptr[DR_EXPORT_COLS], int64_t sz[DR_EXPORT_COLS]) {
  const int64_t n = e->n;
  const int64_t npv = e->pv_entry_off ? e->pv_entry_off[n] : 0;
  const int64_t ntg = e->tags_entry_off ? e->tags_entry_off[n] : 0;
  int k = 0;
#define COL(p, b) do { ptr[k] = (const void*)(p); sz[k] = (int64_t)(b); ++k; } while (0)
  COL(e->path_off, 8 * (n + 1));
  COL(e->path_bytes, e->path_off ? e->path_off[n] : 0);
  COL(e->size, 8 * n);
  COL(e->modification_time, 8 * n);
  COL(e->deletion_timestamp, 8 * n);
  COL(e->deletion_timestamp_valid, n);
  COL(e->extended_file_metadata, n);
  COL(e->stats_off, 8 * (n + 1));
  COL(e->stats_bytes, e->stats_off ? e->stats_off[n] : 0);
  COL(e->stats_null, n);
  COL(e->pv_entry_off, 8 * (n + 1));
  COL(e->pv_null, n);
  COL(e->pv_key_off, 8 * (npv + 1));
  COL(e->pv_key_bytes, e->pv_key_off ? e->pv_key_off[npv] : 0);
  COL(e->pv_val_off, 8 * (npv + 1));
  COL(e->pv_val_bytes, e->pv_val_off ? e->pv_val_off[npv] : 0);
  COL(e->pv_val_null, npv);
  COL(e->tags_entry_off, 8 * (n + 1));
  COL(e->tags_null, n);
  COL(e->tags_key_off, 8 * (ntg + 1));
  COL(e->tags_key_bytes, e->tags_key_off ? e->tags_key_off[ntg] : 0);
  COL(e->tags_val_off, 8 * (ntg + 1));
  COL(e->tags_val_bytes, e->tags_val_off ? e->tags_val_off[ntg] : 0);
  COL(e->tags_val_null, ntg);
#undef COL
}

/* dr_export's columns as direct ByteBuffers, one per column in declaration order (null where a side
 * has no such column, e.g. modificationTime of tombstones). Every buffer's capacity is its exact
 * byte size, so n is pathOff.capacity / 8 - 1 and no extra count crosses. A column over 2^31 - 1
 * bytes (a ByteBuffer's capacity is an int) is refused before any buffer is made. */
static jobjectArray columns(JNIEnv* env, const dr_export* e, const char* too_big) {
  const void* ptr[DR_EXPORT_COLS];
  int64_t sz[DR_EXPORT_COLS];
  column_sizes(e, ptr, sz);
  for (int i = 0; i < DR_EXPORT_COLS; ++i)
    if (ptr[i] && (sz[i] < 0 || sz[i] > 0x7fffffffll)) {
      throw_status(env, DR_E_UNSUPPORTED, too_big);
      return NULL;
    }
  jclass bb = (*env)->FindClass(env, "java/nio/ByteBuffer");
  jobjectArray out = bb ? (*env)->NewObjectArray(env, DR_EXPORT_COLS, bb, NULL) : NULL;
  if (!out) return NULL;
  int failed = 0;
  for (int i = 0; i < DR_EXPORT_COLS && !failed; ++i) {
    jobject b = direct(env, ptr[i], sz[i], &failed);
    if (b && !failed) {
      (*env)->SetObjectArrayElement(env, out, i, b);
      if (pending(env)) failed = 1;
    }
    if (b) (*env)->DeleteLocalRef(env, b);
  }
  return failed ? NULL : out;
}

/* dr_state_export(which), the whole side in one set of buffers (a side whose columns each fit 2 GiB;
 * larger ones go through exportPlan / exportRange). SingleActionColumns (jni/DeltaReplayNative.scala)
 * wraps them into AddFile / RemoveFile rows (D/Snapshot.scala:193-204: allFiles = state.where(add !=
 * null).as[AddFile], tombstones = state.where(remove != null).as[RemoveFile], dataChange = false). */
NATIVE(jobjectArray, export)(JNIEnv* env, jobject self, jlong state, jint which) {
  (void)self;
  dr_export e;
  memset(&e, 0, sizeof e);
  int rc = dr_state_export((dr_state*)(intptr_t)state, which, &e);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  return columns(env, &e, "export: a column over 2^31 - 1 bytes; take the side as row ranges (exportPlan / exportRange)");
}

/* Row ranges of a side whose every column fits maxBytes (<= 2^31 - 1 for direct buffers) and which
 * hold at most maxRows rows: {0, b1, ..., n} (dr_state_export_plan). */
NATIVE(jlongArray, exportPlan)(JNIEnv* env, jobject self, jlong state, jint which, jlong max_rows, jlong max_bytes) {
  (void)self;
  int64_t* b = NULL;
  int64_t nr = 0;
  int rc = max_bytes > 0 ? dr_state_export_plan((dr_state*)(intptr_t)state, which, (int64_t)max_rows,
                                                (uint64_t)max_bytes, &b, &nr)
                         : DR_E_INVALID_ARG;
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  jlongArray out = long_array(env, b, nr + 1);
  dr_free(b);
  return out;
}

/* Rows [lo, hi) of a side as direct buffers with offsets rebased to the range
 * (dr_state_export_range); handleOut(0) receives the range, valid until rangeRelease -- independent
 * of the state, so a partition's rows may outlive the snapshot's uncache. */
NATIVE(jobjectArray, exportRange)(JNIEnv* env, jobject self, jlong state, jint which, jlong lo, jlong hi,
                                  jlongArray handle_out) {
  (void)self;
  if (!handle_out || (*env)->GetArrayLength(env, handle_out) < 1) {
    throw_status(env, DR_E_INVALID_ARG, "exportRange: handleOut must hold one element");
    return NULL;
  }
  dr_range* range = NULL;
  dr_export e;
  memset(&e, 0, sizeof e);
  int rc = dr_state_export_range((dr_state*)(intptr_t)state, which, (int64_t)lo, (int64_t)hi, &range, &e);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  jobjectArray out = columns(env, &e, "exportRange: a column over 2^31 - 1 bytes; plan the ranges with exportPlan");
  if (!out) {
    dr_range_release(range);
    return NULL;
  }
  const jlong h = (jlong)(intptr_t)range;
  (*env)->SetLongArrayRegion(env, handle_out, 0, 1, &h);
  return out;
}

NATIVE(void, rangeRelease)(JNIEnv* env, jobject self, jlong range) {
  (void)env; (void)self;
  dr_range_release((dr_range*)(intptr_t)range);
}

/* ---- scan side ---------------------------------------------------------------------------------- */

/* PartitionFiltering.filesForScan / DeltaLog.filterFileList (D/DeltaLog.scala:500-547): `program` is
 * the shim's lowering of the metadata-only conjuncts, serialised little-endian as
 *   i32 nops,  nops x {i32 opcode, i32 arg}                         (dr_pred_op)
 *   i32 ncols, ncols x {i32 type, i32 name bytes, UTF-8 name}        (partitionSchema, dr_pred_type)
 *   i32 nlits, nlits x {i32 type, u8 null, i64 value, i32 string bytes, UTF-8 string}
 * (DeltaReplayNative.Program.serialize). Returns the selected DR_LIVE positions. */
typedef struct {
  const uint8_t* p;
  const uint8_t* end;
  int ok;
} rd;
static int32_t rd_i32(rd* r) {
  int32_t v = 0;
  if (r->end - r->p < 4) { r->ok = 0; return 0; }
  memcpy(&v, r->p, 4);
  r->p += 4;
  return v;
}
static int64_t rd_i64(rd* r) {
  int64_t v = 0;
  if (r->end - r->p < 8) { r->ok = 0; return 0; }
  memcpy(&v, r->p, 8);
  r->p += 8;
  return v;
}
static const uint8_t* rd_bytes(rd* r, int32_t n) {
  if (n < 0 || r->end - r->p < n) { r->ok = 0; return NULL; }
  const uint8_t* q = r->p;
  r->p += n;
  return q;
}

NATIVE(jlongArray, filter)(JNIEnv* env, jobject self, jlong state, jbyteArray program) {
  (void)self;
  const jsize plen = program ? (*env)->GetArrayLength(env, program) : 0;
  jbyte* prog = program ? (*env)->GetByteArrayElements(env, program, NULL) : NULL;
  rd r = {(const uint8_t*)prog, (const uint8_t*)prog + plen, prog != NULL};
  const int32_t nops = rd_i32(&r);
  dr_pred_op* ops = (dr_pred_op*)calloc((size_t)(nops > 0 ? nops : 0) + 1, sizeof(dr_pred_op));
  for (int32_t i = 0; r.ok && i < nops; ++i) {
    ops[i].opcode = rd_i32(&r);
    ops[i].arg = rd_i32(&r);
  }
  const int32_t ncols = rd_i32(&r);
  const int32_t nc = ncols > 0 ? ncols : 0;
  char** names = (char**)calloc((size_t)nc + 1, sizeof(char*));
  int32_t* types = (int32_t*)calloc((size_t)nc + 1, sizeof(int32_t));
  for (int32_t i = 0; r.ok && i < nc; ++i) {
    types[i] = rd_i32(&r);
    const int32_t len = rd_i32(&r);
    const uint8_t* b = rd_bytes(&r, len);
    if (!b) break;
    names[i] = (char*)malloc((size_t)len + 1);
    memcpy(names[i], b, (size_t)len);
    names[i][len] = 0;
  }
  const int32_t nlits = rd_i32(&r);
  const int32_t nl = nlits > 0 ? nlits : 0;
  int32_t* lt = (int32_t*)calloc((size_t)nl + 1, sizeof(int32_t));
  int64_t* lv = (int64_t*)calloc((size_t)nl + 1, sizeof(int64_t));
  uint8_t* ln = (uint8_t*)calloc((size_t)nl + 1, 1);
  int64_t* soff = (int64_t*)calloc((size_t)nl + 2, sizeof(int64_t));
  uint8_t* sbytes = (uint8_t*)malloc((size_t)plen + 1);
  for (int32_t i = 0; r.ok && i < nl; ++i) {
    lt[i] = rd_i32(&r);
    const uint8_t* nb = rd_bytes(&r, 1);
    ln[i] = nb ? *nb : 1;
    lv[i] = rd_i64(&r);
    const int32_t len = rd_i32(&r);
    const uint8_t* b = rd_bytes(&r, len);
    if (!b) break;
    memcpy(sbytes + soff[i], b, (size_t)len);
    soff[i + 1] = soff[i] + len;
  }
  int64_t* sel = NULL;
  int64_t nsel = 0;
  int rc = DR_E_INVALID_ARG;
  if (r.ok && nops > 0 && r.p == r.end) {
    dr_predicate pred;
    pred.nops = nops; pred.ops = ops;
    pred.ncols = nc; pred.col_names = (const char* const*)names; pred.col_types = types;
    pred.nlits = nl; pred.lit_types = lt; pred.lit_i64 = lv; pred.lit_null = ln;
    pred.lit_str_off = soff; pred.lit_str_bytes = sbytes;
    rc = dr_filter((dr_state*)(intptr_t)state, &pred, &sel, &nsel);
  }
  if (prog) (*env)->ReleaseByteArrayElements(env, program, prog, JNI_ABORT);
  for (int32_t i = 0; i < nc; ++i) free(names[i]);
  free(ops); free(names); free(types); free(lt); free(lv); free(ln); free(soff); free(sbytes);
  if (rc == DR_E_INVALID_ARG && !(r.ok && nops > 0 && r.p == r.end)) {
    throw_status(env, rc, "filter: malformed predicate program");
    return NULL;
  }
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  jlongArray out = long_array(env, sel, nsel);
  dr_free(sel);
  return out;
}

/* DeltaSourceSnapshot.initialFiles' order (D/files/DeltaSourceSnapshot.scala:53-95). */
NATIVE(jlongArray, scanOrder)(JNIEnv* env, jobject self, jlong state) {
  (void)self;
  int64_t* order = NULL;
  int64_t n = 0;
  int rc = dr_state_scan_order((dr_state*)(intptr_t)state, &order, &n);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  jlongArray out = long_array(env, order, n);
  dr_free(order);
  return out;
}

/* TahoeFileIndex.listFiles' groupBy(partitionValues) (D/files/TahoeFileIndex.scala:58-81): {rows in
 * group order, group boundaries}; rows = null groups every live file. */
NATIVE(jobjectArray, partitionGroups)(JNIEnv* env, jobject self, jlong state, jlongArray rows) {
  (void)self;
  const jsize nr = rows ? (*env)->GetArrayLength(env, rows) : 0;
  jlong* rv = rows ? (*env)->GetLongArrayElements(env, rows, NULL) : NULL;
  int64_t *order = NULL, *goff = NULL, ng = 0;
  int rc = dr_state_partition_groups((dr_state*)(intptr_t)state, (const int64_t*)rv, rows ? (int64_t)nr : -1, &order,
                                     &goff, &ng);
  if (rv) (*env)->ReleaseLongArrayElements(env, rows, rv, JNI_ABORT);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  jlongArray o = long_array(env, order, ng ? goff[ng] : 0);
  jlongArray g = o ? long_array(env, goff, ng + 1) : NULL;
  dr_free(order);
  dr_free(goff);
  jclass la = g ? (*env)->FindClass(env, "[J") : NULL;
  jobjectArray out = la ? (*env)->NewObjectArray(env, 2, la, NULL) : NULL;
  if (out) {
    (*env)->SetObjectArrayElement(env, out, 0, o);
    if (!pending(env)) (*env)->SetObjectArrayElement(env, out, 1, g);
  }
  return pending(env) ? NULL : out;
}

/* ---- getChanges (D/DeltaLog.scala:222-238): K1's per-line reading of staged commits -------------- */

/* The dr_lines columns as direct buffers (version, line_off, line_len, kind, flags, path_off, path_len,
 * size, deletion_timestamp, bytes), valid until parsedRelease(handleOut(0)). */
NATIVE(jobjectArray, parseCommits)(JNIEnv* env, jobject self, jlong ctx, jlong staged, jlongArray handle_out) {
  (void)self;
  if (!handle_out || (*env)->GetArrayLength(env, handle_out) < 1) {
    throw_status(env, DR_E_INVALID_ARG, "parseCommits: handleOut must hold one element");
    return NULL;
  }
  dr_parsed* parsed = NULL;
  dr_lines l;
  memset(&l, 0, sizeof l);
  int rc = dr_parse_commits((dr_ctx*)(intptr_t)ctx, (const dr_staged*)(intptr_t)staged, &parsed, &l);
  CHECK_CTX(env, rc, (intptr_t)ctx, NULL);
  const int64_t n = l.n;
  if (n > 0x0fffffffll || l.nbytes > 0x7fffffffull) {
    dr_parsed_release(parsed);
    throw_status(env, DR_E_UNSUPPORTED, "parseCommits: over 2 GiB of commit bytes in one call; stage fewer commits");
    return NULL;
  }
  int failed = 0;
  jobject cols[10];
  cols[0] = direct(env, l.version, 8 * n, &failed);
  cols[1] = direct(env, l.line_off, 8 * n, &failed);
  cols[2] = direct(env, l.line_len, 4 * n, &failed);
  cols[3] = direct(env, l.kind, n, &failed);
  cols[4] = direct(env, l.flags, n, &failed);
  cols[5] = direct(env, l.path_off, 8 * n, &failed);
  cols[6] = direct(env, l.path_len, 4 * n, &failed);
  cols[7] = direct(env, l.size, 8 * n, &failed);
  cols[8] = direct(env, l.deletion_timestamp, 8 * n, &failed);
  cols[9] = direct(env, l.bytes, (int64_t)l.nbytes, &failed);
  jclass bb = failed ? NULL : (*env)->FindClass(env, "java/nio/ByteBuffer");
  jobjectArray out = bb ? (*env)->NewObjectArray(env, 10, bb, NULL) : NULL;
  for (int i = 0; out && i < 10 && !pending(env); ++i) (*env)->SetObjectArrayElement(env, out, i, cols[i]);
  if (!out || pending(env)) {
    dr_parsed_release(parsed);
    return NULL;
  }
  const jlong h = (jlong)(intptr_t)parsed;
  (*env)->SetLongArrayRegion(env, handle_out, 0, 1, &h);
  return out;
}

NATIVE(void, parsedRelease)(JNIEnv* env, jobject self, jlong parsed) {
  (void)env; (void)self;
  dr_parsed_release((dr_parsed*)(intptr_t)parsed);
}

/* ---- multi-GPU: one executor per GPU, RCCL inside the library ---------------- */

NATIVE(jbyteArray, commUniqueId)(JNIEnv* env, jobject self) {
  (void)self;
  uint8_t id[128];
  int rc = dr_comm_unique_id(id);
  if (rc != DR_OK) {
    throw_status(env, rc, "dr_comm_unique_id: RCCL unavailable");
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, 128);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, 128, (const jbyte*)id);
  return out;
}

NATIVE(jlong, commCreate)(JNIEnv* env, jobject self, jlong ctx, jbyteArray id, jint world, jint rank) {
  (void)self;
  if (!id || (*env)->GetArrayLength(env, id) != 128) {
    throw_status(env, DR_E_INVALID_ARG, "commCreate: the id is the 128 bytes of commUniqueId");
    return 0;
  }
  uint8_t buf[128];
  (*env)->GetByteArrayRegion(env, id, 0, 128, (jbyte*)buf);
  dr_comm* comm = NULL;
  int rc = dr_comm_create((dr_ctx*)(intptr_t)ctx, buf, world, rank, &comm);
  CHECK_CTX(env, rc, (intptr_t)ctx, 0);
  return (jlong)(intptr_t)comm;
}

NATIVE(void, commRelease)(JNIEnv* env, jobject self, jlong comm) {
  (void)env; (void)self;
  dr_comm_release((dr_comm*)(intptr_t)comm);
}

/* The shuffle of D/Snapshot.scala:103-104 across GPUs: collective over the communicator's ranks. */
NATIVE(jlong, replaySharded)(JNIEnv* env, jobject self, jlong comm, jlong staged, jlong min_file_retention_ts,
                             jboolean validate) {
  (void)self;
  dr_state* st = NULL;
  int rc = dr_replay_sharded((dr_comm*)(intptr_t)comm, (const dr_staged*)(intptr_t)staged,
                             (int64_t)min_file_retention_ts, validate ? 0u : DR_FLAG_NO_VALIDATION, &st);
  if (rc != DR_OK) {
    throw_status(env, rc, dr_comm_last_error((const dr_comm*)(intptr_t)comm));
    return 0;
  }
  return (jlong)(intptr_t)st;
}

/* ---- Checkpoints.writeCheckpoint (D/Checkpoints.scala:229-365) ---------------------------------- */

/* One complete Parquet part; rowsOut(0) = its rows, rowsOut(1) = its add rows (the caller sums them
 * over the parts and compares with numOfFiles before _last_checkpoint, :325-328). A part larger than
 * a Java array (2 GiB) is refused: write more parts. */
NATIVE(jbyteArray, writeCheckpoint)(JNIEnv* env, jobject self, jlong state, jint part, jint parts, jint opts,
                                    jlong rg_rows, jlongArray rows_out) {
  (void)self;
  uint8_t* bytes = NULL;
  uint64_t len = 0;
  int64_t rows = 0, adds = 0;
  int rc = dr_state_write_checkpoint((dr_state*)(intptr_t)state, part, parts, (uint32_t)opts, (uint64_t)rg_rows,
                                     &bytes, &len, &rows, &adds);
  CHECK_STATE(env, rc, (intptr_t)state, NULL);
  if (len > 0x7fffffffull) {
    dr_free(bytes);
    throw_status(env, DR_E_UNSUPPORTED, "checkpoint part over 2 GiB: write it as more parts");
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, (jsize)len);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)len, (const jbyte*)bytes);
  dr_free(bytes);
  if (!out || pending(env)) return NULL;
  if (rows_out && (*env)->GetArrayLength(env, rows_out) >= 2) {
    const jlong v[2] = {(jlong)rows, (jlong)adds};
    (*env)->SetLongArrayRegion(env, rows_out, 0, 2, v);
  }
  return out;
}
