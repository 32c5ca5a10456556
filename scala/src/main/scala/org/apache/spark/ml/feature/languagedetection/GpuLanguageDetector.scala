package org.apache.spark.ml.feature.languagedetection

import java.nio.charset.StandardCharsets.ISO_8859_1

import org.apache.spark.internal.Logging
import org.apache.spark.ml.Estimator
import org.apache.spark.ml.param.shared.{HasInputCol, HasLabelCol}
import org.apache.spark.ml.param.{Param, ParamMap}
import org.apache.spark.ml.util.Identifiable
import org.apache.spark.sql.types.StructType
import org.apache.spark.sql.{Dataset, SaveMode}

/**
  * Drop-in for the reference's LanguageDetector Estimator (same package, class
  * name, constructors, params, defaults, validation messages and order;
  * LanguageDetector.scala:176-264).  The counting runs on the executors' GPUs
  * (libldgpu.so), see LanguageDetector.computeGramProbabilities.
  */
class LanguageDetector(val uid: String,
                       val supportedLanguages: Seq[String],
                       val gramLengths: Seq[Int],
                       val languageProfileSize: Int)
  extends Estimator[LanguageDetectorModel] with HasInputCol with HasLabelCol {

  def this(supportedLanguages: Seq[String], gramLengths: Seq[Int], languageProfileSize: Int) =
    this(Identifiable.randomUID("LanguageDetector"), supportedLanguages, gramLengths, languageProfileSize)

  setDefault(inputCol -> "fulltext", labelCol -> "lang")

  def setInputCol(value: String): this.type = set(inputCol, value)
  def setLabelCol(value: String): this.type = set(labelCol, value)

  val saveGramsToHDFS = new Param[Option[String]](this, "saveGrams", "Persist the dataset of grams to HDFS")
  def setSaveGramsToHDFS(value: Option[String]): this.type = set(saveGramsToHDFS, value)
  setDefault(saveGramsToHDFS -> None)

  override def transformSchema(schema: StructType): StructType = schema

  override def copy(extra: ParamMap): LanguageDetector =
    copyValues(new LanguageDetector(uid, supportedLanguages, gramLengths, languageProfileSize), extra)

  override def fit(dataset: Dataset[_]): LanguageDetectorModel = {
    import dataset.sparkSession.implicits._
    val data = dataset.select($(labelCol), $(inputCol)).as[(String, String)].cache()
    // the reference's checks, in its order (LanguageDetector.scala:221-238):
    // an unsupported label first (raised inside a job), then a supported
    // language without rows -- one distinct-labels job serves both
    val supported = supportedLanguages.toSet
    val labels = data.map(_._1).distinct()
    labels.foreach { lang =>
      if (!supported.contains(lang))
        throw new Exception(s"Input data contians $lang, but it is not in the list of supported languages")
    }
    val present = labels.collect().toSet
    supportedLanguages.foreach { lang =>
      if (!present.contains(lang))
        throw new Exception(s"No training examples found for language $lang. Provide examples for each language")
    }
    val probabilities =
      LanguageDetector.computeGramProbabilities(data, gramLengths, languageProfileSize, supportedLanguages).cache()
    $(saveGramsToHDFS).foreach(path => LanguageDetector.save(path, probabilities))
    val table = probabilities.collect().toMap
    data.unpersist()
    probabilities.unpersist()
    new LanguageDetectorModel(table, gramLengths, supportedLanguages)
  }
}

/** One gram's nonzero (language, count) pairs, languages ascending: the sparse
  * row of the count table that crosses the shuffle (~1.3 pairs per gram on
  * the fit corpora against nLangs dense Longs). */
final case class SparseCounts(langs: Array[Int], counts: Array[Long]) {
  /** the sum of two rows (a merge of the two sorted language lists) */
  def +(o: SparseCounts): SparseCounts = {
    val l = new Array[Int](langs.length + o.langs.length)
    val c = new Array[Long](l.length)
    var (i, j, k) = (0, 0, 0)
    while (i < langs.length || j < o.langs.length) {
      if (j == o.langs.length || (i < langs.length && langs(i) < o.langs(j))) {
        l(k) = langs(i); c(k) = counts(i); i += 1
      } else if (i == langs.length || o.langs(j) < langs(i)) {
        l(k) = o.langs(j); c(k) = o.counts(j); j += 1
      } else {
        l(k) = langs(i); c(k) = counts(i) + o.counts(j); i += 1; j += 1
      }
      k += 1
    }
    SparseCounts(java.util.Arrays.copyOf(l, k), java.util.Arrays.copyOf(c, k))
  }
}

object LanguageDetector extends Logging {

  /** documents / bytes per ldgpu_count call */
  var batchDocs: Int = 1 << 20
  var batchBytes: Int = 64 << 20
  /** grams per ranged sparse export / import (each range's buffers stay < 2 GiB) */
  var rangeGrams: Long = 1L << 20

  /**
    * computeGramProbabilities (LanguageDetector.scala:145-165) on the GPUs:
    *  1. every partition counts its rows on its executor's GPU (ldgpu_count:
    *     computeGrams + reduceGrams for the partition) and emits one row per
    *     distinct gram: (key, its nonzero (language, count) pairs);
    *  2. one shuffle sums those sparse rows per gram (integer sums: the
    *     reference's counts, bit-exact) -- instead of the reference's L + 1
    *     shuffles of every window record;
    *  3. every partition of the global rows -- each gram in exactly one, with
    *     its global counts, hence its global presence class -- builds its own
    *     top-K table on its GPU (ldgpu_fit_table_size): per language the K best
    *     by (value, then (length, bytes)), which holds every gram of the global
    *     top-K that lives in the partition; it leaves in mask form (key, mask
    *     words, value);
    *  4. the driver keeps, per language, the K best candidates (same order).
    * Ties follow the build's deterministic (length, unsigned bytes) rule where
    * the reference's follow Spark's shuffle order (DESIGN.md, stated
    * divergences); every result satisfies the reference's top-K contract.
    * On Spark with barrier execution, steps 2-4 can instead run inside the
    * library over RCCL (LdgpuNative.countsMerge; INTEGRATION.md).
    */
  def computeGramProbabilities(data: Dataset[(String, String)],
                               gramLengths: Seq[Int],
                               languageProfileSize: Int,
                               supportedLanguages: Seq[String]): Dataset[(Seq[Byte], Array[Double])] = {
    val spark = data.sparkSession
    import spark.implicits._
    val nLangs = supportedLanguages.length
    val index = supportedLanguages.zipWithIndex.toMap
    val grams = gramLengths.toArray
    val (docs, bytes, range) = (batchDocs, batchBytes, rangeGrams)
    val counted = data.rdd.mapPartitions(it => countPartition(it, index, nLangs, grams, docs, bytes, range))
    val global = counted.reduceByKey(_ + _)
    val candidates = global.mapPartitions(it => partitionTopK(it, nLangs, grams, languageProfileSize, range))
    val table = selectTopK(candidates.collect(), nLangs, languageProfileSize)
    spark.createDataset(table.toSeq)
  }

  private def countPartition(it: Iterator[(String, String)], index: Map[String, Int], nLangs: Int,
                             grams: Array[Int], docs: Int, bytes: Int,
                             range: Long): Iterator[(String, SparseCounts)] = {
    if (!it.hasNext) return Iterator.empty
    val ctx = LdgpuNative.context()
    val out = new Array[Long](1)
    LdgpuNative.check(LdgpuNative.countsCreate(ctx, nLangs, grams, 0L, out))
    val counts = out(0)
    val batch = new DocBatch(ctx, docs, bytes)
    try {
      while (it.hasNext) {
        batch.clear()
        while (it.hasNext && !batch.full) {
          val (lang, text) = it.next()
          batch.addFit(text, index.getOrElse(lang, -1))  // rows of other languages are skipped, as reduceGrams does
        }
        LdgpuNative.check(LdgpuNative.count(counts, batch.bytes, batch.offsets, batch.langs, batch.n.toLong))
      }
      exportCounts(counts, range).iterator
    } finally {
      batch.close()
      LdgpuNative.countsDestroy(counts)
    }
  }

  /** (key bytes as an ISO-8859-1 string: one char per byte, a hashable
    * shuffle key; its sparse counts) of every distinct gram of a count table,
    * exported in ranges of at most `range` grams (halved while a range's
    * buffers would pass 1 GiB) */
  private def exportCounts(counts: Long, range: Long): Array[(String, SparseCounts)] = {
    val size = new Array[Long](2)
    LdgpuNative.check(LdgpuNative.countsSize(counts, size))
    val total = size(0)
    val out = new java.util.ArrayList[(String, SparseCounts)](math.min(total, Int.MaxValue - 8).toInt)
    var first = 0L
    while (first < total) {
      var n = math.min(range, total - first)
      val sz = new Array[Long](2)
      LdgpuNative.check(LdgpuNative.countsSparseSize(counts, first, n, sz))
      while (n > 1 && (sz(0) > (1L << 30) || 8L * sz(1) > (1L << 30) || 8L * (n + 1) > (1L << 30))) {
        n = n / 2
        LdgpuNative.check(LdgpuNative.countsSparseSize(counts, first, n, sz))
      }
      val kb = LdgpuNative.direct(sz(0))
      val ko = LdgpuNative.direct(8L * (n + 1))
      val po = LdgpuNative.direct(8L * (n + 1))
      val pl = LdgpuNative.direct(4L * sz(1))
      val pc = LdgpuNative.direct(8L * sz(1))
      LdgpuNative.check(LdgpuNative.countsExportSparse(counts, first, n, kb, ko, po, pl, pc))
      var i = 0
      while (i < n) {
        val (a, b) = (ko.getLong(8 * i).toInt, ko.getLong(8 * (i + 1)).toInt)
        val key = new Array[Byte](b - a)
        kb.position(a)
        kb.get(key)
        val (p0, p1) = (po.getLong(8 * i).toInt, po.getLong(8 * (i + 1)).toInt)
        val langs = new Array[Int](p1 - p0)
        val cnts = new Array[Long](p1 - p0)
        var j = 0
        while (j < langs.length) {
          langs(j) = pl.getInt(4 * (p0 + j))
          cnts(j) = pc.getLong(8 * (p0 + j))
          j += 1
        }
        out.add((new String(key, ISO_8859_1), SparseCounts(langs, cnts)))
        i += 1
      }
      first += n
    }
    out.toArray(new Array[(String, SparseCounts)](out.size))
  }

  /** the partition's global rows into a device table (ranged sparse imports),
    * its top-K table out in mask form: (key, mask words, value) */
  private def partitionTopK(it: Iterator[(String, SparseCounts)], nLangs: Int, grams: Array[Int],
                            profileSize: Int, range: Long): Iterator[(Array[Byte], Array[Long], Double)] = {
    val rows = it.toArray
    if (rows.isEmpty) return Iterator.empty
    val ctx = LdgpuNative.context()
    val out = new Array[Long](1)
    LdgpuNative.check(LdgpuNative.countsCreate(ctx, nLangs, grams, rows.length.toLong, out))
    val counts = out(0)
    try {
      var first = 0
      while (first < rows.length) {
        // the next range: at most `range` rows, its buffers within 1 GiB each
        var n = 0
        var keyBytes = 0L
        var pairs = 0L
        def fits(r: Int): Boolean = n == 0 ||
          (n < range && keyBytes + rows(r)._1.length <= (1L << 30) && 8L * (pairs + rows(r)._2.langs.length) <= (1L << 30))
        while (first + n < rows.length && fits(first + n)) {
          keyBytes += rows(first + n)._1.length
          pairs += rows(first + n)._2.langs.length
          n += 1
        }
        var i = 0
        val kb = LdgpuNative.direct(keyBytes)
        val ko = LdgpuNative.direct(8L * (n + 1))
        val po = LdgpuNative.direct(8L * (n + 1))
        val pl = LdgpuNative.direct(4L * pairs)
        val pc = LdgpuNative.direct(8L * pairs)
        var (ko_, po_) = (0L, 0L)
        ko.putLong(0, 0L)
        po.putLong(0, 0L)
        i = 0
        while (i < n) {
          val (key, sc) = rows(first + i)
          kb.put(key.getBytes(ISO_8859_1))
          ko_ += key.length
          ko.putLong(8 * (i + 1), ko_)
          var j = 0
          while (j < sc.langs.length) {
            pl.putInt(4 * (po_ + j).toInt, sc.langs(j))
            pc.putLong(8 * (po_ + j).toInt, sc.counts(j))
            j += 1
          }
          po_ += sc.langs.length
          po.putLong(8 * (i + 1), po_)
          i += 1
        }
        kb.flip()
        LdgpuNative.check(LdgpuNative.countsAddSparse(counts, n.toLong, kb, ko, po, pl, pc))
        first += n
      }
      val size = new Array[Long](2)
      LdgpuNative.check(LdgpuNative.fitTableSize(counts, profileSize, size))
      val (n, nb) = (size(0), size(1))
      val s = (nLangs + 63) / 64
      val tkb = LdgpuNative.direct(nb)
      val tko = LdgpuNative.direct(8L * (n + 1))
      val tmk = LdgpuNative.direct(8L * n * s)
      val tvl = LdgpuNative.direct(8L * n)
      LdgpuNative.check(LdgpuNative.fitTableExportMasks(counts, tkb, tko, tmk, tvl, n, nb, nLangs))
      Iterator.tabulate(n.toInt) { i =>
        val (a, b) = (tko.getLong(8 * i).toInt, tko.getLong(8 * (i + 1)).toInt)
        val key = new Array[Byte](b - a)
        var j = 0
        while (j < key.length) {
          key(j) = tkb.get(a + j)
          j += 1
        }
        val mask = Array.tabulate(s)(w => tmk.getLong(8 * (i * s + w)))
        (key, mask, tvl.getDouble(8 * i))
      }.toArray.iterator
    } finally {
      LdgpuNative.countsDestroy(counts)
    }
  }

  /** (length, unsigned bytes) order: the build's top-K tie rule */
  private val keyOrder: Ordering[Array[Byte]] = new Ordering[Array[Byte]] {
    override def compare(x: Array[Byte], y: Array[Byte]): Int = {
      if (x.length != y.length) return Integer.compare(x.length, y.length)
      var i = 0
      while (i < x.length) {
        val c = Integer.compare(x(i) & 0xff, y(i) & 0xff)
        if (c != 0) return c
        i += 1
      }
      0
    }
  }

  /** filterTopGrams' final step over the partitions' candidates (mask form):
    * per language the K largest values (ties by key order), the union of the
    * picks with their dense rows (the reference's table type) */
  private def selectTopK(candidates: Array[(Array[Byte], Array[Long], Double)], nLangs: Int,
                         profileSize: Int): Map[Seq[Byte], Array[Double]] = {
    val byKey = candidates.sortWith((a, b) => keyOrder.lt(a._1, b._1))
    def v(i: Int, l: Int): Double = if (((byKey(i)._2(l / 64) >>> (l % 64)) & 1L) != 0L) byKey(i)._3 else 0.0
    val chosen = new java.util.BitSet(byKey.length)
    var l = 0
    while (l < nLangs) {
      val lang = l
      val order = byKey.indices.sortBy(i => -v(i, lang))  // stable: key order among equal values
      order.take(math.max(profileSize, 0)).foreach(i => chosen.set(i))
      l += 1
    }
    byKey.indices.filter(i => chosen.get(i))
      .map(i => (byKey(i)._1.toSeq: Seq[Byte]) -> Array.tabulate(nLangs)(x => v(i, x))).toMap
  }

  def save[T](saveFile: String, ds: Dataset[T]): Unit = {
    logInfo(s"Saving dataset to $saveFile")
    ds.write.format("parquet").mode(SaveMode.Overwrite).save(saveFile)
  }
}
