package org.apache.spark.ml.feature.languagedetection

import java.nio.ByteBuffer
import java.nio.charset.StandardCharsets

import org.apache.spark.unsafe.Platform

/**
  * The gram -> probability-row map as the flat arrays the device table is
  * built from, broadcast by transform (one array per field) instead of a Map of
  * boxed Seq[Byte] keys.  Two forms:
  *  - mask form (every row is one value at a set of languages, 0.0 elsewhere:
  *    every fit-produced row, LanguageDetector.scala:83-87): masks
  *    [n][ceil(L / 64)] and vals [n] -- 8 (S + 1) bytes per row instead of 8 L
  *    (config 5: 10M rows x 200 languages = 16 GB dense, 0.4 GB as masks);
  *  - dense rows [n][nLangs] in supported-language order otherwise, with a
  *    row-length flag: a row whose length differs from the number of
  *    languages is kept with rowOk = 0, and a document that hits it fails as
  *    BLAS.axpy's size check does (LanguageDetectorModel.scala:148-149).
  */
case class PackedTable(keyBytes: Array[Byte], keyOffsets: Array[Long], rows: Array[Double], rowOk: Array[Byte],
                       masks: Array[Long], vals: Array[Double], nLangs: Int) {
  def nRows: Int = keyOffsets.length - 1
  def maskForm: Boolean = masks != null

  def hostBytes: Long =
    keyBytes.length.toLong + 8L * keyOffsets.length +
      (if (maskForm) 8L * masks.length + 8L * vals.length else 8L * rows.length + rowOk.length)

  /** a device table on `ctx` (the executor's GPU) */
  def upload(ctx: Long, gramLengths: Array[Int]): Long = {
    val kb = LdgpuNative.direct(keyBytes.length.toLong)
    kb.put(keyBytes).flip()
    val ko = LdgpuNative.direct(8L * keyOffsets.length)
    ko.asLongBuffer().put(keyOffsets)
    val out = new Array[Long](1)
    if (maskForm) {
      val mk = LdgpuNative.direct(8L * masks.length)
      mk.asLongBuffer().put(masks)
      val vv = LdgpuNative.direct(8L * vals.length)
      vv.asDoubleBuffer().put(vals)
      LdgpuNative.check(LdgpuNative.modelCreateMasks(ctx, nRows.toLong, kb, ko, mk, vv, nLangs, gramLengths, out))
    } else {
      val rw = LdgpuNative.direct(8L * rows.length)
      rw.asDoubleBuffer().put(rows)
      val ok = LdgpuNative.direct(rowOk.length.toLong)
      ok.put(rowOk).flip()
      LdgpuNative.check(LdgpuNative.modelCreate(ctx, nRows.toLong, kb, ko, rw, ok, nLangs, gramLengths, out))
    }
    out(0)
  }
}

object PackedTable {
  def of(map: Map[Seq[Byte], Array[Double]], nLangs: Int): PackedTable = {
    val entries = map.toArray
    val n = entries.length
    val offsets = new Array[Long](n + 1)
    var i = 0
    while (i < n) {
      offsets(i + 1) = offsets(i) + entries(i)._1.length
      i += 1
    }
    val keys = new Array[Byte](offsets(n).toInt)
    i = 0
    while (i < n) {
      entries(i)._1.copyToArray(keys, offsets(i).toInt)
      i += 1
    }
    // mask form when every row has nLangs entries whose non-(+0.0) ones all
    // carry the same finite, nonzero value (bit-exact; per row)
    val s = (nLangs + 63) / 64
    var maskable = n.toLong * s <= Int.MaxValue
    i = 0
    while (i < n && maskable) {
      val row = entries(i)._2
      maskable = row.length == nLangs
      var v = 0L
      var l = 0
      while (l < row.length && maskable) {
        val x = row(l)
        val bits = java.lang.Double.doubleToRawLongBits(x)
        if (bits != 0L) {
          if (x.isNaN || x.isInfinite || x == 0.0) maskable = false
          else if (v == 0L) v = bits
          else maskable = bits == v
        }
        l += 1
      }
      i += 1
    }
    if (maskable) {
      val masks = new Array[Long](n * s)
      val vals = new Array[Double](n)
      i = 0
      while (i < n) {
        val row = entries(i)._2
        var l = 0
        while (l < nLangs) {
          if (java.lang.Double.doubleToRawLongBits(row(l)) != 0L) {
            masks(i * s + l / 64) |= 1L << (l % 64)
            vals(i) = row(l)
          }
          l += 1
        }
        i += 1
      }
      PackedTable(keys, offsets, null, null, masks, vals, nLangs)
    } else {
      val cells = n.toLong * nLangs
      if (cells > Int.MaxValue)
        throw new IllegalArgumentException(s"a dense table of $n rows x $nLangs languages exceeds one JVM array")
      val rows = new Array[Double](cells.toInt)
      val ok = new Array[Byte](n)
      i = 0
      while (i < n) {
        val row = entries(i)._2
        if (row.length == nLangs) {
          System.arraycopy(row, 0, rows, i * nLangs, nLangs)
          ok(i) = 1
        }
        i += 1
      }
      PackedTable(keys, offsets, rows, ok, null, null, nLangs)
    }
  }
}

/**
  * One batch of a partition's documents packed for the C ABI: bytes, int64
  * offsets, int32 language ids (FIT) and int32 labels (SCORE), all direct
  * buffers reused across batches.  Buffers come from ldgpu_host_alloc (pinned
  * host memory) when a context is given, so the library copies them to the
  * GPU without a staging copy.  A batch is full at maxDocs documents or
  * targetBytes bytes (a single larger document grows the byte buffer).
  */
final class DocBatch(ctx: Long, maxDocs: Int, targetBytes: Int) {
  private val pinned = new java.util.IdentityHashMap[ByteBuffer, java.lang.Boolean]()

  private def alloc(bytes: Long): ByteBuffer = {
    val b = if (ctx != 0L) LdgpuNative.hostAlloc(ctx, bytes) else null
    if (b != null) {
      pinned.put(b, java.lang.Boolean.TRUE)
      b.order(java.nio.ByteOrder.nativeOrder())
    } else {
      LdgpuNative.direct(bytes)
    }
  }

  private var byteCap = math.max(targetBytes, 1 << 16)
  // documents are appended with relative bulk puts: bytes.position == used
  var bytes: ByteBuffer = alloc(byteCap.toLong + 16)
  val offsets: ByteBuffer = alloc(8L * (maxDocs + 1))
  val langs: ByteBuffer = alloc(4L * maxDocs)
  val labels: ByteBuffer = alloc(4L * maxDocs)
  var n = 0
  var used = 0
  private var scratch = new Array[Byte](1 << 12)  // one row's bytes, reused
  private var closed = false

  def clear(): Unit = {
    n = 0
    used = 0
    bytes.clear()
    offsets.putLong(0, 0L)
  }

  def full: Boolean = n == maxDocs || used >= targetBytes

  private def ensure(extra: Int): Unit = if (used.toLong + extra > byteCap) {
    val grown = alloc(math.max(2L * byteCap, used.toLong + extra) + 16)
    val old = bytes.duplicate()
    old.position(0).limit(used)
    grown.put(old)  // position = used
    free(bytes)
    bytes = grown
    byteCap = grown.capacity() - 16
  }

  private def scratchOf(len: Int): Array[Byte] = {
    if (scratch.length < len) scratch = new Array[Byte](math.max(len, 2 * scratch.length))
    scratch
  }

  // the first len bytes of b as the next document (one bulk copy)
  private def push(b: Array[Byte], len: Int, lang: Int): Unit = {
    ensure(len)
    bytes.put(b, 0, len)
    used += len
    langs.putInt(4 * n, lang)
    n += 1
    offsets.putLong(8 * n, used.toLong)
  }

  /** SCORE encoding: the low byte of every UTF-16 code unit, as
    * detect(String, ...) does (LanguageDetectorModel.scala:161) -- exactly what
    * String.getBytes(int, int, byte[], int) copies ("each byte receives the 8
    * low-order bits of the corresponding character").  A null text throws
    * NullPointerException there too. */
  def addScore(text: String): Unit = {
    val len = text.length
    val b = scratchOf(len)
    text.getBytes(0, len, b, 0)
    push(b, len, 0)
  }

  /** SCORE encoding straight from Spark's UTF-8 string storage (an
    * InternalRow's UTF8String: base object, offset, byte count): an ASCII row's
    * UTF-8 bytes ARE its low-byte encoding (every UTF-16 unit < 0x80), so they
    * are copied as they are; any other row is decoded and goes through
    * addScore. */
  def addScoreUtf8(base: AnyRef, offset: Long, numBytes: Int, decode: => String): Unit = {
    val b = scratchOf(numBytes)
    Platform.copyMemory(base, offset, b, Platform.BYTE_ARRAY_OFFSET, numBytes)
    var i = 0
    var high = 0
    while (i < numBytes) {
      high |= b(i)
      i += 1
    }
    if (high >= 0) push(b, numBytes, 0)  // no byte with the top bit set: ASCII
    else addScore(decode)
  }

  /** FIT encoding: String.getBytes(UTF-8) (LanguageDetector.scala:37; a lone
    * surrogate becomes '?'); lang = index in supportedLanguages or -1 */
  def addFit(text: String, lang: Int): Unit = {
    val b = text.getBytes(StandardCharsets.UTF_8)
    push(b, b.length, lang)
  }

  def label(i: Int): Int = labels.getInt(4 * i)

  private def free(b: ByteBuffer): Unit = if (b != null && pinned.remove(b) != null) LdgpuNative.hostFree(ctx, b)

  /** idempotent: a task completion listener and the iterator's end may both call it */
  def close(): Unit = if (!closed) {
    closed = true
    Seq(bytes, offsets, langs, labels).foreach(free)
  }
}
