package org.apache.spark.ml.feature.languagedetection.preprocessing

import java.util.Locale

import org.apache.spark.ml.Transformer
import org.apache.spark.ml.param.ParamMap
import org.apache.spark.ml.param.shared.{HasLabelCol, HasOutputCol}
import org.apache.spark.ml.util.{Identifiable, SchemaUtils}
import org.apache.spark.sql.functions.{col, udf}
import org.apache.spark.sql.types.{StringType, StructType}
import org.apache.spark.sql.{DataFrame, Dataset}

/**
 * Host-side drop-in for the reference's LowerCasePreprocessor
 * (LowerCasePreprocessor.scala:19-76): same package, class, constructors,
 * params and defaults (`outputCol` = "fulltext", `labelCol` = "lang").  Not GPU
 * work -- a caller-side cleanup run before fit / transform.
 *
 * Behaviour kept as the reference has it:
 *  - `setInputCol` sets `outputCol` (:32): the text is read from, and written
 *    back to, `outputCol`;
 *  - the text column is dropped and re-appended as the LAST column
 *    (transformSchema :38-42, the row rebuild :63-71);
 *  - each row is lower-cased in the locale of its own label,
 *    `text.toLowerCase(Locale.forLanguageTag(lang))` (:60), so a null text or
 *    label fails the task with a NullPointerException.
 * Written with a UDF over the columns instead of a per-row map of the whole row.
 */
class LowerCasePreprocessor(override val uid: String) extends Transformer with HasOutputCol with HasLabelCol {

  def this() = this(Identifiable.randomUID("LowerCasePreprocessor"))

  setDefault(outputCol -> "fulltext", labelCol -> "lang")

  /** Sets `outputCol`, as the reference does: the column is rewritten in place. */
  def setInputCol(value: String): this.type = set(outputCol, value)

  def setLabelCol(value: String): this.type = set(labelCol, value)

  override def copy(extra: ParamMap): Transformer = defaultCopy(extra)

  override def transformSchema(schema: StructType): StructType =
    SchemaUtils.appendColumn(StructType(schema.fields.filterNot(_.name == $(outputCol))), $(outputCol), StringType,
      nullable = true)

  override def transform(dataset: Dataset[_]): DataFrame = {
    val text = $(outputCol)
    val lowered = udf { (s: String, lang: String) => s.toLowerCase(Locale.forLanguageTag(lang)) }
    val df = dataset.toDF()
    df.schema.fieldIndex(text)        // "Field ... does not exist", as row.fieldIndex
    df.schema.fieldIndex($(labelCol))
    val tmp = LowerCasePreprocessor.freshName(df, text)
    df.withColumn(tmp, lowered(col(text), col($(labelCol))))
      .drop(text)
      .withColumnRenamed(tmp, text)
  }
}

object LowerCasePreprocessor {
  /** a column name not in `df` (the rewritten column's temporary name) */
  private[preprocessing] def freshName(df: DataFrame, base: String): String =
    Iterator.from(0).map(i => s"__ldgpu_${base}_$i").find(n => !df.columns.contains(n)).get
}
