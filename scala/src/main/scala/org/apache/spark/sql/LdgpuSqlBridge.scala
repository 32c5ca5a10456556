package org.apache.spark.sql

import org.apache.spark.rdd.RDD
import org.apache.spark.sql.catalyst.InternalRow
import org.apache.spark.sql.types.StructType

/**
  * The one Spark-internal hook the GPU transform needs: a DataFrame straight
  * from catalyst rows (SparkSession.internalCreateDataFrame is private[sql]).
  * transform reads each row's text as Spark's own UTF-8 bytes (UTF8String)
  * and appends the label, without the Row <-> String conversions of the
  * public Row API.
  */
object LdgpuSqlBridge {
  def internalRows(df: DataFrame): RDD[InternalRow] = df.queryExecution.toRdd

  def fromInternalRows(spark: SparkSession, rows: RDD[InternalRow], schema: StructType): DataFrame =
    spark.internalCreateDataFrame(rows, schema)
}
