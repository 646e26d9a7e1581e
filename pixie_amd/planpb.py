"""px.carnot.planpb message classes for the hot-path subset of plan.proto.

protoc is not available, so the descriptors are declared here field-by-field with the field
numbers of src/carnot/planpb/plan.proto:30-578 and src/shared/types/typespb/types.proto:26-69.
Binary encodings produced with these classes are wire-compatible with the reference's
planpb.Plan.  Used by tests and bench to build plans; the C++ host engine decodes the binary
form itself.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, json_format, text_format
from google.protobuf import message_factory

F = descriptor_pb2.FieldDescriptorProto
_T = {"int64": F.TYPE_INT64, "uint64": F.TYPE_UINT64, "bool": F.TYPE_BOOL, "string": F.TYPE_STRING,
      "double": F.TYPE_DOUBLE, "int32": F.TYPE_INT32}


def _msg(fdp, name, fields, oneofs=None):
    m = fdp.message_type.add()
    m.name = name
    oneof_index = {}
    for o in (oneofs or []):
        oneof_index[o] = len(m.oneof_decl)
        m.oneof_decl.add().name = o
    for spec in fields:
        fname, num, ftype = spec[0], spec[1], spec[2]
        label = spec[3] if len(spec) > 3 else "opt"
        oneof = spec[4] if len(spec) > 4 else None
        f = m.field.add()
        f.name = fname
        f.number = num
        f.label = F.LABEL_REPEATED if label == "rep" else F.LABEL_OPTIONAL
        if ftype in _T:
            f.type = _T[ftype]
        elif ftype.startswith("enum:"):
            f.type = F.TYPE_ENUM
            f.type_name = ftype[5:]
        else:
            f.type = F.TYPE_MESSAGE
            f.type_name = ftype
        if oneof is not None:
            f.oneof_index = oneof_index[oneof]
    return m


def _enum(fdp, name, values):
    e = fdp.enum_type.add()
    e.name = name
    for k, v in values:
        ev = e.value.add()
        ev.name = k
        ev.number = v


def _build():
    pool = descriptor_pool.DescriptorPool()
    types = descriptor_pb2.FileDescriptorProto()
    types.name = "src/shared/types/typespb/types.proto"
    types.package = "px.types"
    types.syntax = "proto3"
    _enum(types, "DataType", [("DATA_TYPE_UNKNOWN", 0), ("BOOLEAN", 1), ("INT64", 2), ("UINT128", 3),
                              ("FLOAT64", 4), ("STRING", 5), ("TIME64NS", 6)])
    _enum(types, "SemanticType", [("ST_UNSPECIFIED", 0), ("ST_NONE", 1), ("ST_TIME_NS", 2), ("ST_UPID", 200),
                                  ("ST_SERVICE_NAME", 300), ("ST_POD_NAME", 400), ("ST_BYTES", 800),
                                  ("ST_PERCENT", 900), ("ST_DURATION_NS", 901), ("ST_QUANTILES", 1000),
                                  ("ST_DURATION_NS_QUANTILES", 1001), ("ST_IP_ADDRESS", 1100),
                                  ("ST_HTTP_RESP_STATUS", 1400)])
    _msg(types, "UInt128", [("low", 1, "uint64"), ("high", 2, "uint64")])
    pool.Add(types)
    from google.protobuf import wrappers_pb2
    wrappers = descriptor_pb2.FileDescriptorProto()
    wrappers_pb2.DESCRIPTOR.CopyToProto(wrappers)
    pool.Add(wrappers)

    p = descriptor_pb2.FileDescriptorProto()
    p.name = "src/carnot/planpb/plan.proto"
    p.package = "px.carnot.planpb"
    p.syntax = "proto3"
    p.dependency.append("src/shared/types/typespb/types.proto")
    p.dependency.append("google/protobuf/wrappers.proto")
    DT = "enum:.px.types.DataType"
    ST = "enum:.px.types.SemanticType"
    _enum(p, "OperatorType", [("OPERATOR_TYPE_UNKNOWN", 0), ("MEMORY_SOURCE_OPERATOR", 1000),
                              ("GRPC_SOURCE_OPERATOR", 1100), ("UDTF_SOURCE_OPERATOR", 1200),
                              ("EMPTY_SOURCE_OPERATOR", 1300), ("MAP_OPERATOR", 2000),
                              ("AGGREGATE_OPERATOR", 2100), ("FILTER_OPERATOR", 2200), ("LIMIT_OPERATOR", 2300),
                              ("UNION_OPERATOR", 2400), ("JOIN_OPERATOR", 2500), ("MEMORY_SINK_OPERATOR", 9000),
                              ("GRPC_SINK_OPERATOR", 9100), ("OTEL_EXPORT_SINK_OPERATOR", 9200)])
    _msg(p, "PlanOptions", [("explain", 2, "bool"), ("analyze", 3, "bool"), ("max_output_rows_per_table", 4, "int64")])
    _msg(p, "Column", [("node", 1, "uint64"), ("index", 2, "uint64")])
    _msg(p, "ScalarValue", [("data_type", 1, DT), ("bool_value", 2, "bool", "opt", "value"),
                            ("int64_value", 3, "int64", "opt", "value"), ("float64_value", 4, "double", "opt", "value"),
                            ("string_value", 5, "string", "opt", "value"), ("time64_ns_value", 6, "int64", "opt", "value"),
                            ("uint128_value", 7, ".px.types.UInt128", "opt", "value")], oneofs=["value"])
    _msg(p, "ScalarFunc", [("name", 1, "string"), ("init_args", 2, ".px.carnot.planpb.ScalarValue", "rep"),
                           ("args", 3, ".px.carnot.planpb.ScalarExpression", "rep"), ("id", 4, "int64"),
                           ("args_data_types", 5, DT, "rep")])
    _msg(p, "ScalarExpression", [("constant", 1, ".px.carnot.planpb.ScalarValue", "opt", "value"),
                                 ("column", 2, ".px.carnot.planpb.Column", "opt", "value"),
                                 ("func", 3, ".px.carnot.planpb.ScalarFunc", "opt", "value")], oneofs=["value"])
    arg = _msg(p, "AggregateExpression", [("name", 3, "string"), ("init_args", 4, ".px.carnot.planpb.ScalarValue", "rep"),
                                          ("args", 5, ".px.carnot.planpb.AggregateExpression.Arg", "rep"), ("id", 6, "int64"),
                                          ("args_data_types", 7, DT, "rep")])
    a = arg.nested_type.add()
    a.name = "Arg"
    a.oneof_decl.add().name = "value"
    for fname, num, tn in [("constant", 1, ".px.carnot.planpb.ScalarValue"), ("column", 2, ".px.carnot.planpb.Column")]:
        f = a.field.add()
        f.name, f.number, f.label, f.type, f.type_name, f.oneof_index = fname, num, F.LABEL_OPTIONAL, F.TYPE_MESSAGE, tn, 0
    _msg(p, "MemorySourceOperator", [("name", 1, "string"), ("column_idxs", 2, "int64", "rep"),
                                     ("column_names", 3, "string", "rep"), ("column_types", 4, DT, "rep"),
                                     ("start_time", 5, ".google.protobuf.Int64Value"),
                                     ("stop_time", 6, ".google.protobuf.Int64Value"),
                                     ("tablet", 7, "string"), ("streaming", 8, "bool")])
    _msg(p, "MemorySinkOperator", [("name", 1, "string"), ("column_types", 2, DT, "rep"),
                                   ("column_names", 3, "string", "rep"), ("column_semantic_types", 4, ST, "rep")])
    rt = _msg(p, "GRPCSinkOperator", [("address", 1, "string"),
                                      ("grpc_source_id", 3, "uint64", "opt", "destination"),
                                      ("output_table", 4, ".px.carnot.planpb.GRPCSinkOperator.ResultTable", "opt", "destination")],
              oneofs=["destination"])
    r = rt.nested_type.add()
    r.name = "ResultTable"
    for fname, num, ftype, lab in [("table_name", 1, F.TYPE_STRING, F.LABEL_OPTIONAL), ("column_types", 2, F.TYPE_ENUM, F.LABEL_REPEATED),
                                   ("column_names", 3, F.TYPE_STRING, F.LABEL_REPEATED),
                                   ("column_semantic_types", 4, F.TYPE_ENUM, F.LABEL_REPEATED)]:
        f = r.field.add()
        f.name, f.number, f.type, f.label = fname, num, ftype, lab
        if num == 2:
            f.type_name = ".px.types.DataType"
        if num == 4:
            f.type_name = ".px.types.SemanticType"
    un = _msg(p, "UnionOperator", [("column_names", 1, "string", "rep"),
                                   ("column_mappings", 2, ".px.carnot.planpb.UnionOperator.ColumnMapping", "rep"),
                                   ("rows_per_batch", 3, "uint64")])
    cm = un.nested_type.add()
    cm.name = "ColumnMapping"
    f = cm.field.add()
    f.name, f.number, f.label, f.type = "column_indexes", 1, F.LABEL_REPEATED, F.TYPE_INT64
    _msg(p, "GRPCSourceOperator", [("column_types", 1, DT, "rep"), ("column_names", 2, "string", "rep")])
    _msg(p, "MapOperator", [("expressions", 1, ".px.carnot.planpb.ScalarExpression", "rep"),
                            ("column_names", 2, "string", "rep")])
    _msg(p, "AggregateOperator", [("values", 1, ".px.carnot.planpb.AggregateExpression", "rep"),
                                  ("groups", 2, ".px.carnot.planpb.Column", "rep"), ("group_names", 3, "string", "rep"),
                                  ("value_names", 4, "string", "rep"), ("windowed", 5, "bool"),
                                  ("partial_agg", 6, "bool"), ("finalize_results", 7, "bool")])
    _msg(p, "FilterOperator", [("expression", 1, ".px.carnot.planpb.ScalarExpression"),
                               ("columns", 2, ".px.carnot.planpb.Column", "rep")])
    _msg(p, "LimitOperator", [("limit", 1, "int64"), ("columns", 2, ".px.carnot.planpb.Column", "rep"),
                              ("abortable_srcs", 3, "uint64", "rep")])
    jo = _msg(p, "JoinOperator", [("type", 1, "enum:.px.carnot.planpb.JoinOperator.JoinType"),
                                  ("equality_conditions", 2, ".px.carnot.planpb.JoinOperator.EqualityCondition", "rep"),
                                  ("output_columns", 3, ".px.carnot.planpb.JoinOperator.ParentColumn", "rep"),
                                  ("column_names", 4, "string", "rep"), ("rows_per_batch", 5, "uint64")])
    je = jo.enum_type.add()
    je.name = "JoinType"
    for k, v in [("INNER", 0), ("LEFT_OUTER", 1), ("FULL_OUTER", 3)]:
        ev = je.value.add()
        ev.name, ev.number = k, v
    for nm, fields in [("EqualityCondition", [("left_column_index", 1), ("right_column_index", 2)]),
                       ("ParentColumn", [("parent_index", 1), ("column_index", 2)])]:
        nt = jo.nested_type.add()
        nt.name = nm
        for fname, num in fields:
            f = nt.field.add()
            f.name, f.number, f.type, f.label = fname, num, F.TYPE_UINT64, F.LABEL_OPTIONAL
    _msg(p, "Operator", [("op_type", 1, "enum:.px.carnot.planpb.OperatorType"),
                         ("mem_source_op", 2, ".px.carnot.planpb.MemorySourceOperator", "opt", "op"),
                         ("map_op", 3, ".px.carnot.planpb.MapOperator", "opt", "op"),
                         ("agg_op", 4, ".px.carnot.planpb.AggregateOperator", "opt", "op"),
                         ("mem_sink_op", 5, ".px.carnot.planpb.MemorySinkOperator", "opt", "op"),
                         ("filter_op", 6, ".px.carnot.planpb.FilterOperator", "opt", "op"),
                         ("limit_op", 7, ".px.carnot.planpb.LimitOperator", "opt", "op"),
                         ("union_op", 8, ".px.carnot.planpb.UnionOperator", "opt", "op"),
                         ("grpc_source_op", 9, ".px.carnot.planpb.GRPCSourceOperator", "opt", "op"),
                         ("join_op", 11, ".px.carnot.planpb.JoinOperator", "opt", "op"),
                         ("grpc_sink_op", 1000, ".px.carnot.planpb.GRPCSinkOperator", "opt", "op")], oneofs=["op"])
    _msg(p, "PlanNode", [("id", 1, "uint64"), ("op", 2, ".px.carnot.planpb.Operator")])
    dag = _msg(p, "DAG", [("nodes", 1, ".px.carnot.planpb.DAG.DAGNode", "rep")])
    dn = dag.nested_type.add()
    dn.name = "DAGNode"
    for fname, num, lab in [("id", 1, F.LABEL_OPTIONAL), ("sorted_children", 3, F.LABEL_REPEATED), ("sorted_parents", 4, F.LABEL_REPEATED)]:
        f = dn.field.add()
        f.name, f.number, f.type, f.label = fname, num, F.TYPE_UINT64, lab
    _msg(p, "PlanFragment", [("id", 1, "uint64"), ("dag", 2, ".px.carnot.planpb.DAG"),
                             ("nodes", 3, ".px.carnot.planpb.PlanNode", "rep")])
    _msg(p, "Plan", [("dag", 1, ".px.carnot.planpb.DAG"), ("nodes", 2, ".px.carnot.planpb.PlanFragment", "rep"),
                     ("plan_options", 4, ".px.carnot.planpb.PlanOptions")])
    pool.Add(p)
    # src/table_store/schemapb/schema.proto:31-79 (RowBatchData, the GRPC transfer payload).
    sc = descriptor_pb2.FileDescriptorProto()
    sc.name = "src/table_store/schemapb/schema.proto"
    sc.package = "px.table_store.schemapb"
    sc.syntax = "proto3"
    sc.dependency.append("src/shared/types/typespb/types.proto")
    for nm, ty in [("BooleanColumn", "bool"), ("Int64Column", "int64"), ("UInt128Column", ".px.types.UInt128"),
                   ("Float64Column", "double"), ("Time64NSColumn", "int64")]:
        _msg(sc, nm, [("data", 1, ty, "rep")])
    sm = sc.message_type.add()
    sm.name = "StringColumn"
    f = sm.field.add()
    f.name, f.number, f.label, f.type = "data", 1, F.LABEL_REPEATED, F.TYPE_BYTES
    S_ = ".px.table_store.schemapb."
    _msg(sc, "Column", [("boolean_data", 1, S_ + "BooleanColumn", "opt", "col_data"),
                        ("int64_data", 2, S_ + "Int64Column", "opt", "col_data"),
                        ("uint128_data", 3, S_ + "UInt128Column", "opt", "col_data"),
                        ("time64ns_data", 4, S_ + "Time64NSColumn", "opt", "col_data"),
                        ("float64_data", 5, S_ + "Float64Column", "opt", "col_data"),
                        ("string_data", 6, S_ + "StringColumn", "opt", "col_data")], oneofs=["col_data"])
    _msg(sc, "RowBatchData", [("cols", 1, S_ + "Column", "rep"), ("num_rows", 2, "int64"), ("eow", 3, "bool"),
                              ("eos", 4, "bool")])
    pool.Add(sc)
    out = {}
    for name in ["Plan", "PlanFragment", "PlanNode", "DAG", "Operator", "MapOperator", "AggregateOperator",
                 "FilterOperator", "LimitOperator", "JoinOperator", "MemorySourceOperator", "MemorySinkOperator", "GRPCSinkOperator",
                 "ScalarExpression", "ScalarValue", "ScalarFunc", "AggregateExpression", "Column", "PlanOptions"]:
        out[name] = message_factory.GetMessageClass(pool.FindMessageTypeByName("px.carnot.planpb." + name))
    out["RowBatchData"] = message_factory.GetMessageClass(pool.FindMessageTypeByName("px.table_store.schemapb.RowBatchData"))
    return out


_CLASSES = _build()
Plan = _CLASSES["Plan"]
PlanFragment = _CLASSES["PlanFragment"]
Operator = _CLASSES["Operator"]
ScalarExpression = _CLASSES["ScalarExpression"]
ScalarValue = _CLASSES["ScalarValue"]
AggregateOperator = _CLASSES["AggregateOperator"]
FilterOperator = _CLASSES["FilterOperator"]
MapOperator = _CLASSES["MapOperator"]
RowBatchData = _CLASSES["RowBatchData"]


def parse_text(cls, text: str):
    msg = cls()
    text_format.Parse(text, msg)
    return msg


def to_json(msg) -> str:
    return json_format.MessageToJson(msg)
