/*
 * JNI shim of BatchRowEncoder (jni/java/org/apache/fory/format/encoder/) over the
 * C-ABI in include/fory_rowfmt.h. Java's buffers are host memory (off-heap
 * MemoryBuffers / direct ByteBuffers, MemoryBuffer.java:287-297), so the shim binds
 * the library's host path (fory_rowfmt_host_*): one context per encoder holds the
 * HIP streams and device chunk slots, and every call pipelines H2D || kernels || D2H.
 * Error codes become the reference's exceptions (Encoders.java:177-225).
 *
 * Build (where a JDK exists):
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       jni/fory_rowfmt_jni.c -Lfury_amd/lib -lfory_rowfmt -o libfory_rowfmt_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "fory_rowfmt.h"

#define CLS(name) Java_org_apache_fory_format_encoder_BatchRowEncoder_##name
#define COLUMN_FIELDS 5 /* ColumnBatch.FIELDS_PER_COLUMN: values, offsets, validity, length, capacity */

static void throw_for(JNIEnv* env, int rc) {
  const char* cls = rc == FORY_ERR_SCHEMA_MISMATCH ? "org/apache/fory/exception/ClassNotCompatibleException"
                    : rc == FORY_ERR_CAPACITY      ? "java/lang/IndexOutOfBoundsException"
                    : rc == FORY_ERR_UNSUPPORTED   ? "java/lang/UnsupportedOperationException"
                    : rc == FORY_ERR_INVALID_ARGUMENT ? "java/lang/IllegalArgumentException"
                                                   : "org/apache/fory/format/encoder/EncoderException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, fory_rowfmt_last_error());
}

static fory_plan* as_plan(jlong p) { return (fory_plan*)(uintptr_t)p; }
static fory_host_ctx* as_ctx(jlong p) { return (fory_host_ctx*)(uintptr_t)p; }

/* ColumnBatch.addresses() -> fory_column[]; caller frees. NULL (exception pending) on failure. */
static fory_column* unpack_array(JNIEnv* env, jlongArray cols, int* ncol) {
  jsize len = (*env)->GetArrayLength(env, cols);
  int n = (int)(len / COLUMN_FIELDS);
  fory_column* out = (fory_column*)calloc(n > 0 ? (size_t)n : 1, sizeof(fory_column));
  if (!out) {
    throw_for(env, FORY_ERR_DEVICE);
    return NULL;
  }
  jlong* a = (*env)->GetLongArrayElements(env, cols, NULL);
  for (int i = 0; i < n; ++i) {
    out[i].values = (void*)(uintptr_t)a[COLUMN_FIELDS * i];
    out[i].offsets = (int32_t*)(uintptr_t)a[COLUMN_FIELDS * i + 1];
    out[i].validity = (uint8_t*)(uintptr_t)a[COLUMN_FIELDS * i + 2];
    out[i].length = a[COLUMN_FIELDS * i + 3];
    out[i].capacity = a[COLUMN_FIELDS * i + 4];
  }
  (*env)->ReleaseLongArrayElements(env, cols, a, JNI_ABORT);
  *ncol = n;
  return out;
}

/* The batch's current columns (an upcall: ColumnBatch.addresses()). */
static fory_column* batch_columns(JNIEnv* env, jobject batch, int* ncol) {
  jclass c = (*env)->GetObjectClass(env, batch);
  jmethodID m = (*env)->GetMethodID(env, c, "addresses", "()[J");
  if (!m) return NULL;
  jlongArray arr = (jlongArray)(*env)->CallObjectMethod(env, batch, m);
  if ((*env)->ExceptionCheck(env) || !arr) return NULL;
  fory_column* cols = unpack_array(env, arr, ncol);
  (*env)->DeleteLocalRef(env, arr);
  return cols;
}

/* ColumnBatch.allocate(counts, bytes) then its new addresses. */
static fory_column* batch_allocate(JNIEnv* env, jobject batch, const int64_t* counts, const int64_t* bytes, int n,
                                   int* ncol) {
  jlongArray jc = (*env)->NewLongArray(env, n);
  jlongArray jb = (*env)->NewLongArray(env, n);
  if (!jc || !jb) return NULL;
  (*env)->SetLongArrayRegion(env, jc, 0, n, (const jlong*)counts);
  (*env)->SetLongArrayRegion(env, jb, 0, n, (const jlong*)bytes);
  jclass c = (*env)->GetObjectClass(env, batch);
  jmethodID m = (*env)->GetMethodID(env, c, "allocate", "([J[J)V");
  if (!m) return NULL;
  (*env)->CallVoidMethod(env, batch, m, jc, jb);
  (*env)->DeleteLocalRef(env, jc);
  (*env)->DeleteLocalRef(env, jb);
  if ((*env)->ExceptionCheck(env)) return NULL;
  return batch_columns(env, batch, ncol);
}

JNIEXPORT jlong JNICALL CLS(nPlanCreate)(JNIEnv* env, jclass cls, jintArray desc) {
  (void)cls;
  jsize n = (*env)->GetArrayLength(env, desc) / 4;
  jint* d = (*env)->GetIntArrayElements(env, desc, NULL);
  fory_plan* plan = NULL;
  int rc = fory_rowfmt_plan_create((const fory_field_desc*)d, (int32_t)n, &plan);  /* 4 x int32 per node */
  (*env)->ReleaseIntArrayElements(env, desc, d, JNI_ABORT);
  if (rc) throw_for(env, rc);
  return (jlong)(uintptr_t)plan;
}

JNIEXPORT void JNICALL CLS(nPlanDestroy)(JNIEnv* env, jclass cls, jlong plan) {
  (void)env, (void)cls;
  fory_rowfmt_plan_destroy(as_plan(plan));
}

JNIEXPORT jlong JNICALL CLS(nSchemaHash)(JNIEnv* env, jclass cls, jlong plan) {
  (void)cls;
  fory_plan_info info;
  int rc = fory_rowfmt_plan_info(as_plan(plan), &info);
  if (rc) throw_for(env, rc);
  return rc ? 0 : (jlong)info.schema_hash;
}

JNIEXPORT jint JNICALL CLS(nRowSize)(JNIEnv* env, jclass cls, jlong plan) {
  (void)cls;
  fory_plan_info info;
  int rc = fory_rowfmt_plan_info(as_plan(plan), &info);
  if (rc) throw_for(env, rc);
  return rc ? -1 : (jint)info.row_size;
}

JNIEXPORT jlong JNICALL CLS(nHostCtxCreate)(JNIEnv* env, jclass cls, jlong plan, jint device, jlong chunk_rows) {
  (void)cls;
  fory_host_ctx* ctx = NULL;
  int rc = fory_rowfmt_host_ctx_create(as_plan(plan), (int32_t)device, (int64_t)chunk_rows, &ctx);
  if (rc) throw_for(env, rc);
  return (jlong)(uintptr_t)ctx;
}

JNIEXPORT void JNICALL CLS(nHostCtxDestroy)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)env, (void)cls;
  fory_rowfmt_host_ctx_destroy(as_ctx(ctx));
}

/* Bytes the batch encodes to (varlen plans): an encode into no room sizes every chunk
   and reports the total with FORY_ERR_CAPACITY (host.cpp: host_encode_var). */
JNIEXPORT jlong JNICALL CLS(nEncodedBytes)(JNIEnv* env, jclass cls, jlong ctx, jlongArray cols, jint n, jint frame) {
  (void)cls;
  int ncol = 0;
  fory_column* hc = unpack_array(env, cols, &ncol);
  if (!hc) return 0;
  int64_t total = 0;
  int rc = fory_rowfmt_host_encode_var(as_ctx(ctx), hc, n, frame, NULL, 0, NULL, &total);
  free(hc);
  if (rc && rc != FORY_ERR_CAPACITY) {
    throw_for(env, rc);
    return 0;
  }
  return (jlong)total;
}

/* The exact bytes of each <= max_window window of the batch's frames (varlen plans): the
   device sizes every row (an encode into no room reports the row offsets with
   FORY_ERR_CAPACITY), fory_rowfmt_split_windows places whole frames greedily. */
JNIEXPORT jlongArray JNICALL CLS(nWindowBytes)(JNIEnv* env, jclass cls, jlong ctx, jlongArray cols, jint n, jint frame,
                                               jlong max_window) {
  (void)cls;
  int ncol = 0;
  fory_column* hc = unpack_array(env, cols, &ncol);
  if (!hc) return NULL;
  int64_t* offs = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
  int64_t* first = (int64_t*)calloc((size_t)n + 2, sizeof(int64_t));
  int64_t total = 0;
  int32_t nw = 0;
  int rc = offs && first ? fory_rowfmt_host_encode_var(as_ctx(ctx), hc, n, frame, NULL, 0, offs, &total)
                         : FORY_ERR_DEVICE;
  if (rc == FORY_ERR_CAPACITY) rc = FORY_OK;  /* sizes only: no room given */
  if (!rc) rc = fory_rowfmt_split_windows(offs, 0, n, (int64_t)max_window, n > 0 ? n : 1, first, &nw);
  jlongArray out = NULL;
  if (!rc) {
    const int32_t k = nw > 0 ? nw : 1;
    out = (*env)->NewLongArray(env, k);
    if (out) {
      for (int32_t w = 0; w < k; ++w) {
        const jlong b = nw > 0 ? (jlong)(offs[first[w + 1]] - offs[first[w]]) : 0;
        (*env)->SetLongArrayRegion(env, out, w, 1, &b);
      }
    }
  }
  free(hc);
  free(offs);
  free(first);
  if (rc) throw_for(env, rc);
  return out;
}

JNIEXPORT void JNICALL CLS(nEncodeWindows)(JNIEnv* env, jclass cls, jlong ctx, jlongArray cols, jint n, jint frame,
                                           jlongArray addrs, jlongArray caps, jlongArray bytes) {
  (void)cls;
  int ncol = 0;
  fory_column* hc = unpack_array(env, cols, &ncol);
  if (!hc) return;
  jsize nw = (*env)->GetArrayLength(env, addrs);
  int64_t* got = (int64_t*)calloc(nw > 0 ? (size_t)nw : 1, sizeof(int64_t));
  jlong* a = (*env)->GetLongArrayElements(env, addrs, NULL);
  jlong* k = (*env)->GetLongArrayElements(env, caps, NULL);
  void** ptrs = (void**)calloc(nw > 0 ? (size_t)nw : 1, sizeof(void*));
  for (jsize w = 0; w < nw; ++w) ptrs[w] = (void*)(uintptr_t)a[w];
  int rc = got && ptrs ? fory_rowfmt_host_encode_windows(as_ctx(ctx), hc, n, frame, (void* const*)ptrs,
                                                          (const int64_t*)k, (int32_t)nw, NULL, got)
                       : FORY_ERR_DEVICE;
  (*env)->ReleaseLongArrayElements(env, addrs, a, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, caps, k, JNI_ABORT);
  if (!rc) (*env)->SetLongArrayRegion(env, bytes, 0, nw, (const jlong*)got);
  free(hc);
  free(got);
  free(ptrs);
  if (rc) throw_for(env, rc);  /* FORY_ERR_CAPACITY -> IndexOutOfBoundsException */
}

JNIEXPORT jlong JNICALL CLS(nEncodeVar)(JNIEnv* env, jclass cls, jlong ctx, jlongArray cols, jint n, jint frame,
                                        jlong out_addr, jlong out_cap, jlongArray row_offsets) {
  (void)cls;
  int ncol = 0;
  fory_column* hc = unpack_array(env, cols, &ncol);
  if (!hc) return 0;
  int64_t* offs = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
  int64_t total = 0;
  int rc = offs ? fory_rowfmt_host_encode_var(as_ctx(ctx), hc, n, frame, (void*)(uintptr_t)out_addr, out_cap, offs,
                                              &total)
                : FORY_ERR_DEVICE;
  if (!rc) (*env)->SetLongArrayRegion(env, row_offsets, 0, n + 1, (const jlong*)offs);
  free(hc);
  free(offs);
  if (rc) throw_for(env, rc);
  return (jlong)total;
}

/* N x decode(MemoryBuffer) over the frames alone (varlen plans): device frame index +
   sizes, the receiver's columns sized by an upcall, then the values. */
JNIEXPORT jlong JNICALL CLS(nDecodeStream)(JNIEnv* env, jclass cls, jlong ctx, jlong in_addr, jlong in_len, jint n,
                                           jobject out) {
  (void)cls;
  int ncol = 0;
  fory_column* cur = batch_columns(env, out, &ncol);
  if (!cur) return 0;
  int64_t* counts = (int64_t*)calloc((size_t)ncol + 1, sizeof(int64_t));
  int64_t* bytes = (int64_t*)calloc((size_t)ncol + 1, sizeof(int64_t));
  int64_t consumed = 0;
  int rc = counts && bytes ? fory_rowfmt_host_decode_stream_sizes(as_ctx(ctx), (const void*)(uintptr_t)in_addr,
                                                                  in_len, n, counts, bytes, &consumed)
                           : FORY_ERR_DEVICE;
  fory_column* cols = NULL;
  if (!rc) {
    cols = batch_allocate(env, out, counts, bytes, ncol, &ncol);
    rc = cols ? fory_rowfmt_host_decode_var(as_ctx(ctx), cols) : -1;  /* -1: a Java exception is pending */
  }
  free(cur);
  free(cols);
  free(counts);
  free(bytes);
  if (rc > 0) throw_for(env, rc);  /* SCHEMA_MISMATCH -> ClassNotCompatibleException; CORRUPT */
  return (jlong)consumed;
}

/* N x decode(MemoryBuffer) of a fixed-width plan: every frame is row_size + 12 bytes
   (fory_rowfmt_host_decode checks each frame's size and schema hash on the device). */
JNIEXPORT void JNICALL CLS(nDecodeFixed)(JNIEnv* env, jclass cls, jlong ctx, jlong in_addr, jlong in_len, jint n,
                                         jint frame, jobject out) {
  (void)cls;
  int ncol = 0;
  fory_column* cur = batch_columns(env, out, &ncol);
  if (!cur) return;
  int64_t* counts = (int64_t*)calloc((size_t)ncol + 1, sizeof(int64_t));
  int64_t* bytes = (int64_t*)calloc((size_t)ncol + 1, sizeof(int64_t));
  fory_column* cols = NULL;
  int rc = FORY_ERR_DEVICE;
  if (counts && bytes) {
    for (int i = 0; i < ncol; ++i) counts[i] = n;
    cols = batch_allocate(env, out, counts, bytes, ncol, &ncol);
    rc = cols ? fory_rowfmt_host_decode(as_ctx(ctx), (const void*)(uintptr_t)in_addr, in_len, n, frame, cols) : -1;
  }
  free(cur);
  free(cols);
  free(counts);
  free(bytes);
  if (rc > 0) throw_for(env, rc);
}

/* N x decode(MemoryBuffer) with the frame offsets: one pipelined call into the
   receiver's columns; a batch that does not fit reports its sizes, the columns grow
   (upcall) and the call repeats. */
JNIEXPORT void JNICALL CLS(nDecodeInto)(JNIEnv* env, jclass cls, jlong ctx, jlong in_addr, jlongArray offs, jint n,
                                        jint frame, jobject out) {
  (void)cls;
  int ncol = 0;
  fory_column* cols = batch_columns(env, out, &ncol);
  if (!cols) return;
  int64_t* counts = (int64_t*)calloc((size_t)ncol + 1, sizeof(int64_t));
  int64_t* bytes = (int64_t*)calloc((size_t)ncol + 1, sizeof(int64_t));
  jlong* o = (*env)->GetLongArrayElements(env, offs, NULL);
  int rc = counts && bytes ? fory_rowfmt_host_decode_var_into(as_ctx(ctx), (const void*)(uintptr_t)in_addr,
                                                              (const int64_t*)o, n, frame, cols, counts, bytes)
                           : FORY_ERR_DEVICE;
  if (rc == FORY_ERR_CAPACITY) {
    free(cols);
    cols = batch_allocate(env, out, counts, bytes, ncol, &ncol);
    rc = cols ? fory_rowfmt_host_decode_var_into(as_ctx(ctx), (const void*)(uintptr_t)in_addr, (const int64_t*)o, n,
                                                 frame, cols, counts, bytes)
              : -1;
  }
  (*env)->ReleaseLongArrayElements(env, offs, o, JNI_ABORT);
  free(cols);
  free(counts);
  free(bytes);
  if (rc > 0) throw_for(env, rc);
}

JNIEXPORT void JNICALL CLS(nRegister)(JNIEnv* env, jclass cls, jlong addr, jlong nbytes) {
  (void)cls;
  int rc = fory_rowfmt_host_register((void*)(uintptr_t)addr, nbytes);
  if (rc) throw_for(env, rc);
}

JNIEXPORT void JNICALL CLS(nUnregister)(JNIEnv* env, jclass cls, jlong addr) {
  (void)cls;
  int rc = fory_rowfmt_host_unregister((void*)(uintptr_t)addr);
  if (rc) throw_for(env, rc);
}
