/* Minimal declarations of the JNI types and JNIEnv functions jni/fory_rowfmt_jni.c uses,
   with the JNI specification's C signatures — ONLY so that a CPU test can syntax-check
   the shim against include/fory_rowfmt.h where no JDK (and so no real jni.h) exists. */
#ifndef FORY_TEST_JNI_STUB_H_
#define FORY_TEST_JNI_STUB_H_
#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef jint jsize;
struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jlongArray;
struct _jmethodID;
typedef struct _jmethodID* jmethodID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
  jclass (*GetObjectClass)(JNIEnv* env, jobject obj);
  jmethodID (*GetMethodID)(JNIEnv* env, jclass clazz, const char* name, const char* sig);
  jobject (*CallObjectMethod)(JNIEnv* env, jobject obj, jmethodID methodID, ...);
  void (*CallVoidMethod)(JNIEnv* env, jobject obj, jmethodID methodID, ...);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
  jint* (*GetIntArrayElements)(JNIEnv* env, jintArray array, jboolean* isCopy);
  jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
  void (*ReleaseIntArrayElements)(JNIEnv* env, jintArray array, jint* elems, jint mode);
  void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
};
#endif
