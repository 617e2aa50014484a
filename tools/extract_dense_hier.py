"""Dev tool (run in the build container only; /root/reference does not exist on the GPU box).
Also reads hier_model_struct.build (train_hier_networks.py:338-530) with ``path=REF_HIER`` and
dense_model_struct.build (train_dense_networks.py:223-408) with ``path=REF_DENSE``.

Reads dense_hier_model_struct.build (/root/reference/train_dense_hier_networks.py:338-2382) as an
AST -- the file as a whole is Python 2 and does not parse, the build body does -- and writes the
layer graph it constructs as data: one record per op in build order, with static shapes
propagated from a [N,128,128,1] input.  Used by tests/test_dense_hier.py to pin the package's own
restatement (monkey-pose_amd/dense_hier_graph.py) against the reference's structure, and to
record the digest committed in tests/golden/dense_hier_graph.json.

  python tools/extract_dense_hier.py [out.json]
"""
import ast
import json
import sys

REF = "/root/reference/train_dense_hier_networks.py"
REF_HIER = "/root/reference/train_hier_networks.py"   # hier_model_struct.build (338-530), same vocabulary
REF_DENSE = "/root/reference/train_dense_networks.py"  # dense_model_struct.build (223-408)
REF_CNN = "/root/reference/train_cnn_networks_hgru.py"   # cnn_model_struct.build (639-673): cls="cnn_model_struct"


def _src_build(path=REF, cls=None):
    lines = open(path).read().split("\n")
    first = 0 if cls is None else next(i for i, l in enumerate(lines) if l.startswith(f"class {cls}"))
    start = next(i for i in range(first, len(lines)) if lines[i].strip().startswith("def build(self,depth,output_shape"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith("def "))
    body = "\n".join(l[4:] if l.startswith("    ") else l for l in lines[start:end])
    return ast.parse(body).body[0], start + 1


def _attr(node):
    if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) and node.value.id == "self":
        return node.attr
    raise ValueError(ast.dump(node))


def _const(node):
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.Mult):
        return _const(node.left) * _const(node.right)
    return ast.literal_eval(node)


def extract(heads=(108, 39, 39, 39, 39, 36), path=REF, cls=None):
    fn, line0 = _src_build(path, cls)
    shapes = {"lr_input": (128, 128, 1)}
    alias = {}
    ops = []
    outs = dict(zip(("output_shape", "P_shape", "R_shape", "M_shape", "I_shape", "T_shape"), heads))

    def t(node):
        if isinstance(node, ast.Name) and node.id == "input_image":
            return "lr_input"
        n = _attr(node)
        return alias.get(n, n)

    def size_of(node):
        if isinstance(node, ast.Name):
            return outs[node.id]
        return _const(node)

    for st in fn.body:
        if isinstance(st, ast.If) or isinstance(st, ast.Expr):
            continue  # dropout under train_mode==True / print
        if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Name):
            continue  # input_image = tf.identity(depth)
        assert isinstance(st, ast.Assign), ast.dump(st)
        dst = _attr(st.targets[0])
        call = st.value
        f = call.func
        fname = f.attr if isinstance(f, ast.Attribute) else f.id
        owner = ast.unparse(f.value) if isinstance(f, ast.Attribute) else ""
        kw = {k.arg: k.value for k in call.keywords}
        line = line0 + st.lineno - 1
        if fname == "conv_layer":
            a = call.args
            src = t(a[0])
            cin_lit = a[1]
            cout = _const(a[2])
            name = _const(a[3]) if len(a) > 3 else _const(kw["name"])
            k = _const(kw.get("filter_size", ast.Constant(3)))
            stride = _const(kw["stride"])[1] if "stride" in kw else 1
            H, W, C = shapes[src]
            if not isinstance(cin_lit, ast.Call):
                assert _const(cin_lit) == C, (line, name, _const(cin_lit), C)
            Ho, Wo = -(-H // stride), -(-W // stride)
            shapes[dst] = (Ho, Wo, cout)
            ops.append(dict(op="conv", out=dst, name=name, src=src, k=k, stride=stride, cin=C, cout=cout, line=line))
        elif fname in ("max_pool", "avg_pool", "max_pool_4"):
            src = t(call.args[0])
            H, W, C = shapes[src]
            p = 4 if fname == "max_pool_4" else 2
            shapes[dst] = (-(-H // p), -(-W // p), C)
            ops.append(dict(op="avgpool" if fname == "avg_pool" else "maxpool", out=dst, src=src, k=p, line=line))
        elif fname == "concat" and owner == "tf":
            srcs = [t(e) for e in call.args[0].elts]
            hw = {shapes[s][:2] for s in srcs}
            assert len(hw) == 1, (line, dst)
            shapes[dst] = (*hw.pop(), sum(shapes[s][-1] for s in srcs))
            ops.append(dict(op="concat", out=dst, srcs=srcs, line=line))
        elif fname == "fc_layer":
            a = call.args
            src = t(a[0])
            H, W, C = shapes[src]
            K = H * W * C
            if not isinstance(a[1], ast.Call):
                assert _const(a[1]) == K, (line, a[3], K)
            cout = size_of(a[2])
            shapes[dst] = (1, 1, cout)
            ops.append(dict(op="fc", out=dst, name=_const(a[3]), src=src, cin=K, cout=cout, line=line))
        elif fname == "relu" and owner == "tf.nn":
            src = t(call.args[0])
            shapes[dst] = shapes[src]
            ops.append(dict(op="relu", out=dst, src=src, line=line))
        elif fname == "identity" and owner == "tf":
            src = t(call.args[0])
            alias[dst] = src
            shapes[dst] = shapes[src]
            ops.append(dict(op="identity", out=dst, src=src, line=line))
        else:
            raise ValueError(f"unhandled op at {line}: {fname}")
    names = [o["name"] for o in ops if "name" in o]
    assert len(names) == len(set(names)), "duplicate variable scopes"
    return ops, {k: list(v) for k, v in shapes.items()}


if __name__ == "__main__":
    ops, shapes = extract()
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/dense_hier_graph.json"
    json.dump(dict(ops=ops, shapes=shapes), open(out, "w"), indent=0)
    import collections
    print(collections.Counter(o["op"] for o in ops), "->", out)
