package org.apache.spark.ml.feature.languagedetection

import java.nio.{ByteBuffer, ByteOrder}
import java.util.concurrent.ConcurrentHashMap

/**
  * JNI bindings of libldgpu.so (include/ldgpu.h) through libldgpu_jni.so
  * (jni/ldgpu_jni.c).  Every buffer argument is a DIRECT ByteBuffer in native
  * byte order; handles are the C pointers as Longs.  A non-zero status turns
  * into the JVM exception the reference raises for the same condition
  * (LdgpuNative.check).
  *
  * Per executor JVM: one context per device and one device table per
  * broadcast table (LanguageDetectorModel.scala:222 broadcasts the map once
  * per transform), shared by the executor's task threads -- every C entry
  * point is thread-safe and concurrent scoring calls run on their own
  * streams.
  */
object LdgpuNative {
  System.loadLibrary("ldgpu_jni")

  // ---- C ABI (status codes of enum ldgpu_status)
  val OK = 0
  val EINVAL = 1
  val EROWLEN = 2
  val ENOMEM = 3
  val EDEVICE = 4
  val EUNSUPPORTED = 5
  val ENODEV = 6

  @native def lastError(): String
  @native def ctxCreate(device: Int, out: Array[Long]): Int
  @native def hostAlloc(ctx: Long, bytes: Long): ByteBuffer          // pinned, direct; null on failure
  @native def hostFree(ctx: Long, buf: ByteBuffer): Int
  @native def modelCreate(ctx: Long, nRows: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, rows: ByteBuffer,
                          rowOk: ByteBuffer, nLangs: Int, gramLengths: Array[Int], out: Array[Long]): Int
  @native def modelDestroy(model: Long): Int
  @native def score(model: Long, bytes: ByteBuffer, offsets: ByteBuffer, nDocs: Long, labels: ByteBuffer,
                    scores: ByteBuffer): Int
  @native def countsCreate(ctx: Long, nLangs: Int, gramLengths: Array[Int], capacityHint: Long,
                           out: Array[Long]): Int
  @native def countsDestroy(counts: Long): Int
  @native def count(counts: Long, bytes: ByteBuffer, offsets: ByteBuffer, docLang: ByteBuffer, nDocs: Long): Int
  /** out(0) = distinct grams, out(1) = their total key bytes */
  @native def countsSize(counts: Long, out: Array[Long]): Int
  @native def countsExport(counts: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, counts_ : ByteBuffer): Int
  @native def countsAdd(counts: Long, n: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, rows: ByteBuffer): Int
  /** out(0) = table rows, out(1) = their total key bytes */
  @native def fitTableSize(counts: Long, profileSize: Int, out: Array[Long]): Int
  @native def fitTableExport(counts: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, rows: ByteBuffer): Int
  // multi-GPU merge (Spark with barrier execution: one task per GPU)
  @native def commUniqueId(): Array[Byte]
  @native def commCreateRccl(ctx: Long, id: Array[Byte], rank: Int, world: Int, out: Array[Long]): Int
  @native def commDestroy(comm: Long): Int
  @native def countsMerge(counts: Long, comm: Long): Int

  /** The reference's exception for each failure class: a wrong-length row
    * hit (BLAS.axpy's require) and n <= 0 (sliding's require) are
    * IllegalArgumentException, allocation failures OutOfMemoryError. */
  def check(status: Int): Unit = status match {
    case OK => ()
    case EINVAL | EROWLEN => throw new IllegalArgumentException(lastError())
    case ENOMEM => throw new OutOfMemoryError(lastError())
    case EUNSUPPORTED => throw new UnsupportedOperationException(lastError())
    case _ => throw new RuntimeException(s"libldgpu: ${lastError()}")
  }

  def direct(bytes: Long): ByteBuffer =
    ByteBuffer.allocateDirect(math.max(bytes, 1L).toInt).order(ByteOrder.nativeOrder())

  /** The executor's GPU: executors are pinned one per GPU (HIP_VISIBLE_DEVICES),
    * so device 0 unless LDGPU_DEVICE says otherwise. */
  def defaultDevice: Int = sys.env.get("LDGPU_DEVICE").map(_.toInt).getOrElse(0)

  private val contexts = new ConcurrentHashMap[Integer, java.lang.Long]()

  def context(device: Int = defaultDevice): Long = {
    val have = contexts.get(device)
    if (have != null) have.longValue
    else contexts.synchronized {
      val again = contexts.get(device)
      if (again != null) again.longValue
      else {
        val out = new Array[Long](1)
        check(ctxCreate(device, out))
        contexts.put(device, out(0))
        out(0)
      }
    }
  }

  // device tables of this executor, keyed by the broadcast that carries them
  private val models = new ConcurrentHashMap[java.lang.Long, java.lang.Long]()

  def model(broadcastId: Long, table: PackedTable, gramLengths: Array[Int]): Long = {
    val have = models.get(broadcastId)
    if (have != null) have.longValue
    else models.synchronized {
      val again = models.get(broadcastId)
      if (again != null) again.longValue
      else {
        val h = table.upload(context(), gramLengths)
        models.put(broadcastId, h)
        h
      }
    }
  }

  def releaseModel(broadcastId: Long): Unit = {
    val h = models.remove(broadcastId)
    if (h != null) modelDestroy(h.longValue)
  }
}
