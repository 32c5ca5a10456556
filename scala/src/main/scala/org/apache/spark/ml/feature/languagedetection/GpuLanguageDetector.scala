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

object LanguageDetector extends Logging {

  /** documents / bytes per ldgpu_count call */
  var batchDocs: Int = 1 << 20
  var batchBytes: Int = 64 << 20

  /**
    * computeGramProbabilities (LanguageDetector.scala:145-165) on the GPUs:
    *  1. every partition counts its rows on its executor's GPU (ldgpu_count:
    *     computeGrams + reduceGrams for the partition) and emits one row per
    *     distinct gram: (key, counts[L]);
    *  2. one shuffle sums those rows per gram (integer sums: the reference's
    *     counts, bit-exact) -- instead of the reference's L + 1 shuffles of
    *     every window record;
    *  3. every partition of the global rows -- each gram in exactly one, with
    *     its global counts, hence its global presence class -- builds its own
    *     top-K table on its GPU (ldgpu_fit_table_size): per language the K best
    *     by (value, then (length, bytes)), which holds every gram of the global
    *     top-K that lives in the partition;
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
    val (docs, bytes) = (batchDocs, batchBytes)
    val counted = data.rdd.mapPartitions(it => countPartition(it, index, nLangs, grams, docs, bytes))
    val global = counted.reduceByKey { (a, b) =>
      val s = new Array[Long](a.length)
      var l = 0
      while (l < a.length) {
        s(l) = a(l) + b(l)
        l += 1
      }
      s
    }
    val candidates = global.mapPartitions(it => partitionTopK(it, nLangs, grams, languageProfileSize))
    val table = selectTopK(candidates.collect(), nLangs, languageProfileSize)
    spark.createDataset(table.toSeq)
  }

  private def countPartition(it: Iterator[(String, String)], index: Map[String, Int], nLangs: Int,
                             grams: Array[Int], docs: Int, bytes: Int): Iterator[(String, Array[Long])] = {
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
      exportCounts(counts, nLangs).iterator
    } finally {
      batch.close()
      LdgpuNative.countsDestroy(counts)
    }
  }

  /** (key bytes as an ISO-8859-1 string: one char per byte, a hashable
    * shuffle key; counts[L]) of every distinct gram of a count table */
  private def exportCounts(counts: Long, nLangs: Int): Array[(String, Array[Long])] = {
    val size = new Array[Long](2)
    LdgpuNative.check(LdgpuNative.countsSize(counts, size))
    val (n, nb) = (size(0).toInt, size(1))
    val kb = LdgpuNative.direct(nb)
    val ko = LdgpuNative.direct(8L * (n + 1))
    val cs = LdgpuNative.direct(8L * n * nLangs)
    LdgpuNative.check(LdgpuNative.countsExport(counts, kb, ko, cs))
    Array.tabulate(n) { i =>
      val (a, b) = (ko.getLong(8 * i).toInt, ko.getLong(8 * (i + 1)).toInt)
      val key = new Array[Byte](b - a)
      var j = 0
      while (j < key.length) {
        key(j) = kb.get(a + j)
        j += 1
      }
      val row = new Array[Long](nLangs)
      var l = 0
      while (l < nLangs) {
        row(l) = cs.getLong(8 * (i * nLangs + l))
        l += 1
      }
      (new String(key, ISO_8859_1), row)
    }
  }

  private def partitionTopK(it: Iterator[(String, Array[Long])], nLangs: Int, grams: Array[Int],
                            profileSize: Int): Iterator[(Array[Byte], Array[Double])] = {
    val rows = it.toArray
    if (rows.isEmpty) return Iterator.empty
    val ctx = LdgpuNative.context()
    val out = new Array[Long](1)
    LdgpuNative.check(LdgpuNative.countsCreate(ctx, nLangs, grams, rows.length.toLong, out))
    val counts = out(0)
    try {
      val keys = rows.map(_._1.getBytes(ISO_8859_1))
      val ko = LdgpuNative.direct(8L * (keys.length + 1))
      var off = 0L
      ko.putLong(0, 0L)
      keys.indices.foreach { i =>
        off += keys(i).length
        ko.putLong(8 * (i + 1), off)
      }
      val kb = LdgpuNative.direct(off)
      keys.foreach(k => kb.put(k))
      kb.flip()
      val cs = LdgpuNative.direct(8L * rows.length * nLangs)
      rows.iterator.zipWithIndex.foreach { case ((_, row), i) =>
        var l = 0
        while (l < nLangs) {
          cs.putLong(8 * (i * nLangs + l), row(l))
          l += 1
        }
      }
      LdgpuNative.check(LdgpuNative.countsAdd(counts, rows.length.toLong, kb, ko, cs))
      val size = new Array[Long](2)
      LdgpuNative.check(LdgpuNative.fitTableSize(counts, profileSize, size))
      val (n, nb) = (size(0).toInt, size(1))
      val tkb = LdgpuNative.direct(nb)
      val tko = LdgpuNative.direct(8L * (n + 1))
      val trw = LdgpuNative.direct(8L * n * nLangs)
      LdgpuNative.check(LdgpuNative.fitTableExport(counts, tkb, tko, trw))
      Array.tabulate(n) { i =>
        val (a, b) = (tko.getLong(8 * i).toInt, tko.getLong(8 * (i + 1)).toInt)
        val key = Array.tabulate(b - a)(j => tkb.get(a + j))
        (key, Array.tabulate(nLangs)(l => trw.getDouble(8 * (i * nLangs + l))))
      }.iterator
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

  /** filterTopGrams' final step over the partitions' candidates: per
    * language the K largest values (ties by key order), union of the picks */
  private def selectTopK(candidates: Array[(Array[Byte], Array[Double])], nLangs: Int,
                         profileSize: Int): Map[Seq[Byte], Array[Double]] = {
    val byKey = candidates.sortWith((a, b) => keyOrder.lt(a._1, b._1))
    val chosen = new java.util.BitSet(byKey.length)
    var l = 0
    while (l < nLangs) {
      val lang = l
      val order = byKey.indices.sortBy(i => -byKey(i)._2(lang))  // stable: key order among equal values
      order.take(math.max(profileSize, 0)).foreach(i => chosen.set(i))
      l += 1
    }
    byKey.indices.filter(i => chosen.get(i)).map(i => (byKey(i)._1.toSeq: Seq[Byte]) -> byKey(i)._2).toMap
  }

  def save[T](saveFile: String, ds: Dataset[T]): Unit = {
    logInfo(s"Saving dataset to $saveFile")
    ds.write.format("parquet").mode(SaveMode.Overwrite).save(saveFile)
  }
}
