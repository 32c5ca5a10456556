// The Scala drop-in for the reference's Spark ML API (same package and class
// names), over libldgpu.so through jni/libldgpu_jni.so.  Spark 2.2 / Scala
// 2.11 like the reference (its build.sbt); executors need libldgpu.so and
// libldgpu_jni.so on java.library.path (spark.executor.extraLibraryPath).
name := "spark-languagedetector-amd"
version := "0.2.0"
scalaVersion := "2.11.11"
libraryDependencies ++= Seq(
  "org.apache.spark" %% "spark-core" % "2.2.0" % "provided",
  "org.apache.spark" %% "spark-sql" % "2.2.0" % "provided",
  "org.apache.spark" %% "spark-mllib" % "2.2.0" % "provided"
)
