/*
 * capnp_packed_jni.c -- JNI glue between org.capnproto.gpu.PackedGpu and the
 * C ABI of include/capnp_packed.h.  Built where a JDK exists (this image has
 * none; INTEGRATION.md gives the command):
 *
 *   cc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *      -I../../../include capnp_packed_jni.c \
 *      -L../../lib -lcapnp_packed_hip -Wl,-rpath,'$ORIGIN' -o libcapnp_packed_jni.so
 *
 * Buffers: direct ByteBuffers are passed zero-copy (GetDirectBufferAddress;
 * DIRECT allocation exists in the reference, DefaultAllocator.java:56-62);
 * heap buffers are pinned with Get/ReleasePrimitiveArrayCritical.  Status
 * codes become the reference's exceptions: decode errors ->
 * org.capnproto.DecodeException (DecodeException.java:24-27), device / memory
 * errors -> java.io.IOException.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "capnp_packed.h"

static void throw_status(JNIEnv *env, int st) {
  const char *cls = (st == CPK_ETRUNC || st == CPK_EOVERRUN || st == CPK_ETRAILING ||
                     st == CPK_EINVAL)
                        ? "org/capnproto/DecodeException"
                        : "java/io/IOException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, cpk_status_string(st));
}

/* long PackedGpu.nativeCreate(int device) */
JNIEXPORT jlong JNICALL Java_org_capnproto_gpu_PackedGpu_nativeCreate(JNIEnv *env, jclass k,
                                                                       jint device) {
  (void)k;
  cpk_ctx ctx = NULL;
  int st = cpk_ctx_create(device, &ctx);
  if (st != CPK_OK) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeDestroy(JNIEnv *env, jclass k,
                                                                      jlong h) {
  (void)env;
  (void)k;
  cpk_ctx_destroy((cpk_ctx)(intptr_t)h);
}

JNIEXPORT jlong JNICALL Java_org_capnproto_gpu_PackedGpu_nativeCapacity(JNIEnv *env, jclass k,
                                                                        jlongArray segWordOff) {
  (void)k;
  jsize n1 = (*env)->GetArrayLength(env, segWordOff);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  uint64_t cap = cpk_batch_packed_capacity((const uint64_t *)swo, (uint32_t)(n1 - 1));
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  return (jlong)cap;
}

/* Encodes n pieces held back to back in `in` (direct buffer, position 0):
 * piece i = words [segWordOff[i], segWordOff[i+1]).  Writes the packed stream
 * to `out` (direct) and the piece offsets to outOff[n+1].  Same bytes as n
 * PackedOutputStream.write calls (PackedOutputStream.java:35-205). */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeEncode(
    JNIEnv *env, jclass k, jlong h, jobject in, jlongArray segWordOff, jobject out,
    jlongArray outOff) {
  (void)k;
  void *pin = (*env)->GetDirectBufferAddress(env, in);
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  jlong cap = (*env)->GetDirectBufferCapacity(env, out);
  if (!pin || !pout) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  jsize n1 = (*env)->GetArrayLength(env, segWordOff);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  jlong *off = (*env)->GetLongArrayElements(env, outOff, NULL);
  int st = cpk_encode_host((cpk_ctx)(intptr_t)h, pin, (const uint64_t *)swo, (uint32_t)(n1 - 1),
                           pout, (uint64_t)cap, (uint64_t *)off);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, outOff, off, 0);
  if (st != CPK_OK) throw_status(env, st);
}

/* Decodes n pieces: piece i's packed bytes are packed[inOff[i]..inOff[i+1])
 * and it fills words [segWordOff[i], segWordOff[i+1]) of `out`.  Throws the
 * first piece's error (DecodeException) like PackedInputStream.read. */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeDecode(
    JNIEnv *env, jclass k, jlong h, jobject packed, jlongArray inOff, jlongArray segWordOff,
    jobject out) {
  (void)k;
  void *ppk = (*env)->GetDirectBufferAddress(env, packed);
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  if (!ppk || !pout) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  jsize n1 = (*env)->GetArrayLength(env, segWordOff);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  jlong *io = (*env)->GetLongArrayElements(env, inOff, NULL);
  int32_t *status = (int32_t *)calloc((size_t)(n1 > 1 ? n1 - 1 : 1), sizeof(int32_t));
  int st = cpk_decode_host((cpk_ctx)(intptr_t)h, ppk, (const uint64_t *)io,
                           (const uint64_t *)swo, (uint32_t)(n1 - 1), pout, status);
  free(status);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, inOff, io, JNI_ABORT);
  if (st != CPK_OK) throw_status(env, st);
}
