/* Minimal stand-in for <jni.h>, for tests only (this image has no JDK):
 * the types, macros and the JNIEnv function-table entries that
 * capnproto-java_amd/java/jni/capnp_packed_jni.c uses, with the JNI
 * specification's signatures.  The table layout is this file's own (a fake
 * environment, tests/jni/fake_env.c, fills it); the glue only ever calls
 * through (*env)->Name(env, ...), so compiling and running it against this
 * table exercises exactly its own logic.  A real build uses the JDK's
 * header. */
#ifndef CPK_TEST_JNI_H
#define CPK_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
#define JNI_COMMIT 1

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jlongArray;
typedef jarray jintArray;
typedef jarray jobjectArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv *env, const char *name);
  jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
  void (*DeleteLocalRef)(JNIEnv *env, jobject obj);
  jsize (*GetArrayLength)(JNIEnv *env, jarray array);
  jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
  jlong *(*GetLongArrayElements)(JNIEnv *env, jlongArray array, jboolean *isCopy);
  void (*ReleaseLongArrayElements)(JNIEnv *env, jlongArray array, jlong *elems, jint mode);
  jint *(*GetIntArrayElements)(JNIEnv *env, jintArray array, jboolean *isCopy);
  void (*ReleaseIntArrayElements)(JNIEnv *env, jintArray array, jint *elems, jint mode);
  void (*SetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, const jlong *buf);
  void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};

#endif
