// Package graphing: the drop-in for the reference's graphing package
// (at15/nemo graphing/*.go).  This file replaces the Cypher-carrying files
// (helpers.go, pre-post-prov.go, preprocessing.go, prototype.go,
// differential-provenance.go, the two query functions of corrections.go,
// extensions.go); diagrams.go, hazard-analysis.go and corrections.go's string
// synthesis stay.  Every Neo4j round trip is a call into libnemohip's C ABI
// (include/nemohip.h).  See go/README.md for where the file goes and the one
// refactor of corrections.go it needs.
package graphing

/*
#cgo CFLAGS: -I${SRCDIR}/../third_party/nemohip/include
#cgo LDFLAGS: -L${SRCDIR}/../third_party/nemohip/nemo_amd -lnemohip -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
#include <stdlib.h>
#include "nemohip.h"
*/
import "C"

import (
	"fmt"
	"sort"
	"strings"
	"unsafe"

	"github.com/awalterschulze/gographviz"
	"github.com/johnnadratowski/golang-neo4j-bolt-driver/structures/graph"

	fi "github.com/numbleroot/nemo/faultinjectors"
)

// Neo4J keeps its name and its exported field so main.go:95 (&gr.Neo4J{}) is
// untouched; it no longer talks to Neo4j (pre-post-prov.go:16-20).
type Neo4J struct {
	Runs []*fi.Run

	ctx     *C.nemo_ctx
	tables  []string          // interned table names, id = index
	tableID map[string]uint32
	labels  []string          // interned labels (exact interning, never a hash)
	labelID map[string]uint32
	runIdx  map[uint]int      // Run.Iteration -> run index (graph 2r = pre, 2r+1 = post)
	graphs  []*provGraph      // per graph g, node-index order
	chains  map[int][][2]uint32 // accepted @next chains per graph: (head, tail) by k
	red     *reduction          // last nemo_protos_finalize
}

// One loaded provenance graph: loadProv creates goals first, then rules
// (pre-post-prov.go:27-58,90-118), so local node i < len(Goals) is goal i.
type provGraph struct {
	iter     uint
	cond     string
	goals    []fi.Goal
	rules    []fi.Rule
	src, dst []uint32 // the loaded edges (local indices): the raw graph's relationships
}

func (p *provGraph) n() int { return len(p.goals) + len(p.rules) }

type reduction struct {
	achieved, nRuns uint32
	inter, union    []uint32
	preHolds        uint64
}

func (n *Neo4J) err(rc C.int) error {
	if rc == C.NEMO_OK {
		return nil
	}
	return fmt.Errorf("%s", C.GoString(C.nemo_last_error(n.ctx)))
}

func (n *Neo4J) intern(tab *[]string, ids map[string]uint32, s string) uint32 {
	if id, ok := ids[s]; ok {
		return id
	}
	id := uint32(len(*tab))
	*tab = append(*tab, s)
	ids[s] = id
	return id
}

func typeClass(t string) uint32 {
	switch t {
	case "next":
		return C.NEMO_TYPE_NEXT
	case "async":
		return C.NEMO_TYPE_ASYNC
	}
	return C.NEMO_TYPE_OTHER
}

// ---- helpers.go ---------------------------------------------------------------

// InitGraphDB (helpers.go:17-55): no docker-compose, no 10 s sleep, no Bolt;
// boltURI is accepted and ignored.  One node context over every GPU of the
// node: the corpus is run-sharded inside the library (include/nemohip.h).
func (n *Neo4J) InitGraphDB(boltURI string, runs []*fi.Run) error {
	if rc := C.nemo_ctx_create_node(0, nil, &n.ctx); rc != C.NEMO_OK {
		return fmt.Errorf("nemo_ctx_create_node: status %d", int(rc))
	}
	n.Runs = runs
	n.tableID, n.labelID = map[string]uint32{}, map[string]uint32{}
	n.runIdx = map[uint]int{}
	for r, run := range runs {
		n.runIdx[run.Iteration] = r
	}
	return nil
}

// CloseDB (helpers.go:58-86).
func (n *Neo4J) CloseDB() error {
	C.nemo_ctx_destroy(n.ctx)
	n.ctx = nil
	return nil
}

// ---- pre-post-prov.go -----------------------------------------------------------

// LoadRawProvenance (pre-post-prov.go:247-285): loadProv for every run's pre
// and post graph as interning into one nemo_corpus, one load (CSR build, the
// reference's validations, Kahn levels on the device), one markConditionHolds.
func (n *Neo4J) LoadRawProvenance() error {
	R := len(n.Runs)
	iters := make([]C.uint32_t, R)
	nodeOff, edgeOff := []C.uint64_t{0}, []C.uint64_t{0}
	var words, labels, ranks, src, dst []C.uint32_t
	n.graphs = n.graphs[:0]
	for r, run := range n.Runs {
		iters[r] = C.uint32_t(run.Iteration)
		for _, cond := range []string{"pre", "post"} {
			prov := run.PreProv
			if cond == "post" {
				prov = run.PostProv
			}
			if prov == nil {
				prov = &fi.ProvData{}
			}
			g := &provGraph{iter: run.Iteration, cond: cond, goals: prov.Goals, rules: prov.Rules}
			index := make(map[string]uint32, g.n())
			ids := make([]string, 0, g.n())
			for _, goal := range prov.Goals {
				index[goal.ID] = uint32(len(ids))
				ids = append(ids, goal.ID)
				words = append(words, C.uint32_t(n.intern(&n.tables, n.tableID, goal.Table)))
				labels = append(labels, C.uint32_t(n.intern(&n.labels, n.labelID, goal.Label)))
			}
			// Goal.id IS UNIQUE (pre-post-prov.go:66-81): a duplicate is not a second node
			nGoals := len(index)
			if nGoals != len(prov.Goals) {
				return fmt.Errorf("Run %d: inserted number of goals (%d) does not equal number of antecedent provenance goals (%d)", run.Iteration, nGoals, len(prov.Goals))
			}
			for _, rule := range prov.Rules {
				index[rule.ID] = uint32(len(ids))
				ids = append(ids, rule.ID)
				w := C.NEMO_NODE_RULE | typeClass(rule.Type)<<C.NEMO_TYPE_SHIFT | n.intern(&n.tables, n.tableID, rule.Table)
				words = append(words, C.uint32_t(w))
				labels = append(labels, C.uint32_t(n.intern(&n.labels, n.labelID, rule.Label)))
			}
			if len(index)-nGoals != len(prov.Rules) { // Rule.id IS UNIQUE (:126-141)
				return fmt.Errorf("Run %d: inserted number of rules (%d) does not equal number of antecedent provenance rules (%d)", run.Iteration, len(index)-nGoals, len(prov.Rules))
			}
			// rank of each ID inside the graph: the canonical @next tie-break (DESIGN.md §1)
			order := make([]int, len(ids))
			for i := range order {
				order[i] = i
			}
			sort.Slice(order, func(a, b int) bool { return ids[order[a]] < ids[order[b]] })
			rank := make([]C.uint32_t, len(ids))
			for pos, i := range order {
				rank[i] = C.uint32_t(pos)
			}
			ranks = append(ranks, rank...)
			// edges: direction by strings.Contains(From, "goal") (:173); a missing
			// endpoint or a duplicate creates no relationship, and the count check
			// of :208-210 then fails exactly as the reference's does
			seen := map[[2]uint32]bool{}
			created := 0
			for _, e := range prov.Edges {
				u, okU := index[e.From]
				v, okV := index[e.To]
				fromGoal := strings.Contains(e.From, "goal")
				if !okU || !okV || (int(u) < len(prov.Goals)) != fromGoal || (int(v) < len(prov.Goals)) == fromGoal ||
					seen[[2]uint32{u, v}] {
					continue
				}
				seen[[2]uint32{u, v}] = true
				src = append(src, C.uint32_t(u))
				dst = append(dst, C.uint32_t(v))
				g.src = append(g.src, u)
				g.dst = append(g.dst, v)
				created++
			}
			if created != len(prov.Edges) {
				return fmt.Errorf("Run %d: inserted number of edges (%d) does not equal number of antecedent provenance edges (%d)",
					run.Iteration, created, len(prov.Edges))
			}
			nodeOff = append(nodeOff, C.uint64_t(len(words)))
			edgeOff = append(edgeOff, C.uint64_t(len(src)))
			n.graphs = append(n.graphs, g)
		}
	}
	n.intern(&n.tables, n.tableID, "pre")
	n.intern(&n.tables, n.tableID, "post")
	var corpus C.nemo_corpus
	corpus.n_runs = C.uint32_t(R)
	corpus.n_tables = C.uint32_t(len(n.tables))
	corpus.table_pre = C.uint32_t(n.tableID["pre"])
	corpus.table_post = C.uint32_t(n.tableID["post"])
	corpus.iteration = cArray(iters)
	corpus.node_off, corpus.edge_off = cArray(nodeOff), cArray(edgeOff)
	corpus.node_word, corpus.label, corpus.id_rank = cArray(words), cArray(labels), cArray(ranks)
	corpus.edge_src, corpus.edge_dst = cArray(src), cArray(dst)
	defer freeCorpus(&corpus)
	if err := n.err(C.nemo_load_corpus(n.ctx, &corpus)); err != nil {
		return err
	}
	return n.err(C.nemo_mark_holds(n.ctx))
}

// cArray copies a Go slice to C memory (cgo forbids Go pointers to Go pointers).
func cArray[T any](s []T) *T {
	if len(s) == 0 {
		return nil
	}
	var z T
	p := (*T)(C.malloc(C.size_t(len(s)) * C.size_t(unsafe.Sizeof(z))))
	copy(unsafe.Slice(p, len(s)), s)
	return p
}

func freeCorpus(c *C.nemo_corpus) {
	for _, p := range []unsafe.Pointer{unsafe.Pointer(c.iteration), unsafe.Pointer(c.node_off),
		unsafe.Pointer(c.edge_off), unsafe.Pointer(c.node_word), unsafe.Pointer(c.label),
		unsafe.Pointer(c.id_rank), unsafe.Pointer(c.edge_src), unsafe.Pointer(c.edge_dst)} {
		C.free(p)
	}
}

// ---- preprocessing.go -------------------------------------------------------------

// SimplifyProv (preprocessing.go:351-387): cleanCopyProv + collapseNextChains
// of every loaded run on the device; the accepted chains come back once.
func (n *Neo4J) SimplifyProv(iters []uint) error {
	for _, it := range iters {
		if _, ok := n.runIdx[it]; !ok {
			return fmt.Errorf("SimplifyProv: run %d was not loaded", it)
		}
	}
	if err := n.err(C.nemo_simplify(n.ctx)); err != nil {
		return err
	}
	var cnt C.uint64_t
	if err := n.err(C.nemo_fetch_chains(n.ctx, nil, 0, &cnt)); err != nil {
		return err
	}
	ch := make([]C.nemo_chain, int(cnt)+1)
	if err := n.err(C.nemo_fetch_chains(n.ctx, &ch[0], cnt, &cnt)); err != nil {
		return err
	}
	n.chains = map[int][][2]uint32{}
	for _, c := range ch[:cnt] { // ordered by (graph, k)
		g := int(c.graph)
		n.chains[g] = append(n.chains[g], [2]uint32{uint32(c.head), uint32(c.tail)})
	}
	return nil
}

// ---- node properties (what loadProv stored, plus the device flags) ---------------

func rewriteRun(id string, old, new uint) string { // the `id`:"run_<old> rewrite (preprocessing.go:33-45)
	pfx := fmt.Sprintf("run_%d", old)
	if strings.HasPrefix(id, pfx) {
		return fmt.Sprintf("run_%d", new) + id[len(pfx):]
	}
	return id
}

// node returns the bolt-driver graph.Node createDOT reads (diagrams.go:41-83):
// labels "Goal"/"Rule", properties id, label, table, type, condition_holds,
// time.  run != nil re-prefixes the ID like the clean (1000+i) and diff
// (2000+f) copies.  Local index V_g+k is collapsed rule k (preprocessing.go:249-252).
func (n *Neo4J) node(g int, i uint32, flags []uint8, run *uint) graph.Node {
	pg := n.graphs[g]
	V := uint32(pg.n())
	if i >= V {
		k := i - V
		head := n.chains[g][k][0]
		table := pg.rules[int(head)-len(pg.goals)].Table
		lab := table + "_collapsed"
		return graph.Node{Labels: []string{"Rule"}, Properties: map[string]interface{}{
			"id": fmt.Sprintf("run_%d_%s_%s_%d", 1000+pg.iter, pg.cond, lab, k), "label": lab,
			"table": table, "type": "collapsed"}}
	}
	if int(i) < len(pg.goals) {
		goal := pg.goals[i]
		id := goal.ID
		if run != nil {
			id = rewriteRun(id, pg.iter, *run)
		}
		return graph.Node{Labels: []string{"Goal"}, Properties: map[string]interface{}{
			"id": id, "label": goal.Label, "table": goal.Table, "time": goal.Time,
			"condition_holds": flags[i]&C.NEMO_F_HOLDS != 0}}
	}
	rule := pg.rules[int(i)-len(pg.goals)]
	id := rule.ID
	if run != nil {
		id = rewriteRun(id, pg.iter, *run)
	}
	return graph.Node{Labels: []string{"Rule"}, Properties: map[string]interface{}{
		"id": id, "label": rule.Label, "table": rule.Table, "type": rule.Type}}
}

func (n *Neo4J) flags(g int) ([]uint8, error) {
	f := make([]uint8, n.graphs[g].n()+1)
	if err := n.err(C.nemo_fetch_node_flags(n.ctx, C.uint32_t(g), C.uint32_t(g+1), (*C.uint8_t)(&f[0]), C.uint64_t(len(f)))); err != nil {
		return nil, err
	}
	return f, nil
}

// paths turns pulled slot `slot` of graph g into the []graph.Path rows
// createDOT / createDiffDot consume, in (source, target) order.
func (n *Neo4J) paths(slot uint32, g int, run *uint) ([]graph.Path, error) {
	var cnt C.uint64_t
	if err := n.err(C.nemo_fetch_pulled(n.ctx, C.uint32_t(slot), nil, nil, 0, &cnt)); err != nil {
		return nil, err
	}
	s, d := make([]uint32, cnt+1), make([]uint32, cnt+1)
	if err := n.err(C.nemo_fetch_pulled(n.ctx, C.uint32_t(slot), (*C.uint32_t)(&s[0]), (*C.uint32_t)(&d[0]), cnt, &cnt)); err != nil {
		return nil, err
	}
	return n.edgeRows(s[:cnt], d[:cnt], g, run)
}

// rawPaths: the rows of raw graph g (run i, pre-post-prov.go:298-301) are its
// loaded edges, which the binding holds, so no device pull is needed.
func (n *Neo4J) rawPaths(g int) ([]graph.Path, error) {
	return n.edgeRows(n.graphs[g].src, n.graphs[g].dst, g, nil)
}

func (n *Neo4J) edgeRows(s, d []uint32, g int, run *uint) ([]graph.Path, error) {
	cnt := len(s)
	idx := make([]int, cnt)
	for i := range idx {
		idx[i] = i
	}
	sort.Slice(idx, func(a, b int) bool {
		if s[idx[a]] != s[idx[b]] {
			return s[idx[a]] < s[idx[b]]
		}
		return d[idx[a]] < d[idx[b]]
	})
	fl, err := n.flags(g)
	if err != nil {
		return nil, err
	}
	out := make([]graph.Path, 0, cnt)
	for _, j := range idx {
		out = append(out, graph.Path{Nodes: []graph.Node{n.node(g, s[j], fl, run), n.node(g, d[j], fl, run)},
			Relationships: []graph.UnboundRelationship{{Type: "DUETO"}}})
	}
	return out, nil
}

// PullPrePostProv (pre-post-prov.go:288-459): raw graphs (run i) and
// simplified graphs (run 1000+i) of every run, through createDOT (unchanged).
func (n *Neo4J) PullPrePostProv() ([]*gographviz.Graph, []*gographviz.Graph, []*gographviz.Graph, []*gographviz.Graph, error) {
	R := len(n.Runs)
	pre, post := make([]*gographviz.Graph, R), make([]*gographviz.Graph, R)
	preC, postC := make([]*gographviz.Graph, R), make([]*gographviz.Graph, R)
	var err error
	var rows []graph.Path
	for r := 0; r < R; r++ {
		if rows, err = n.rawPaths(2 * r); err != nil {
			return nil, nil, nil, nil, err
		}
		if pre[r], err = createDOT(rows, "pre"); err != nil {
			return nil, nil, nil, nil, err
		}
		if rows, err = n.rawPaths(2*r + 1); err != nil {
			return nil, nil, nil, nil, err
		}
		if post[r], err = createDOT(rows, "post"); err != nil {
			return nil, nil, nil, nil, err
		}
	}
	if err = n.err(C.nemo_pull_edges(n.ctx, 1)); err != nil {
		return nil, nil, nil, nil, err
	}
	for r := 0; r < R; r++ {
		clean := 1000 + n.Runs[r].Iteration
		if rows, err = n.paths(uint32(2*r), 2*r, &clean); err != nil {
			return nil, nil, nil, nil, err
		}
		if preC[r], err = createDOT(rows, "pre"); err != nil {
			return nil, nil, nil, nil, err
		}
		if rows, err = n.paths(uint32(2*r+1), 2*r+1, &clean); err != nil {
			return nil, nil, nil, nil, err
		}
		if postC[r], err = createDOT(rows, "post"); err != nil {
			return nil, nil, nil, nil, err
		}
	}
	return pre, post, preC, postC, nil
}

// ---- prototype.go -------------------------------------------------------------------

func (n *Neo4J) reduce(success []uint) (*reduction, error) {
	s := make([]C.uint32_t, len(success)+1)
	for i, it := range success {
		s[i] = C.uint32_t(it)
	}
	if err := n.err(C.nemo_protos_partial(n.ctx, &s[0], C.size_t(len(success)), nil)); err != nil {
		return nil, err
	}
	T := len(n.tables)
	inter, uni := make([]C.uint32_t, T+1), make([]C.uint32_t, T+1)
	var achvd, ni, nu, nr C.uint32_t
	var ph C.uint64_t
	if err := n.err(C.nemo_protos_finalize(n.ctx, nil, &achvd, &inter[0], &ni, &uni[0], &nu, &ph, &nr)); err != nil {
		return nil, err
	}
	red := &reduction{achieved: uint32(achvd), nRuns: uint32(nr), preHolds: uint64(ph)}
	for _, t := range inter[:ni] {
		red.inter = append(red.inter, uint32(t))
	}
	for _, t := range uni[:nu] {
		red.union = append(red.union, uint32(t))
	}
	n.red = red
	return red, nil
}

func (n *Neo4J) tableNames(ids []uint32) []string {
	out := make([]string, len(ids))
	for i, t := range ids {
		out[i] = n.tables[t]
	}
	return out
}

func codeWrap(ts []string) []string { // prototype.go:245-251
	out := make([]string, len(ts))
	for i, t := range ts {
		out[i] = fmt.Sprintf("<code>%s</code>", t)
	}
	return out
}

// missingFrom (prototype.go:141-206): proto entries absent from the failed
// run's simplified post graph, in proto order, wrapped in <code> (:196).
func (n *Neo4J) missingFrom(proto []uint32, failedIter uint) ([]string, error) {
	p := make([]C.uint32_t, len(proto)+1)
	for i, t := range proto {
		p[i] = C.uint32_t(t)
	}
	out := make([]C.uint32_t, len(proto)+1)
	var cnt C.uint32_t
	if err := n.err(C.nemo_missing_from(n.ctx, C.uint32_t(failedIter), &p[0], C.uint32_t(len(proto)), &out[0], &cnt)); err != nil {
		return nil, err
	}
	ids := make([]uint32, cnt)
	for i := range ids {
		ids[i] = uint32(out[i])
	}
	return codeWrap(n.tableNames(ids)), nil
}

// CreatePrototypes (prototype.go:209-256): extractProtos on the device,
// inter/union from the (all-reduced) vector, missingFrom per failed run,
// <code> wrapping after the missing computation (:245-251).
func (n *Neo4J) CreatePrototypes(iters []uint, failedIters []uint) ([]string, [][]string, []string, [][]string, error) {
	if len(iters) == 0 { // the reference indexes iterProv[0] (prototype.go:80) and panics
		return nil, nil, nil, nil, fmt.Errorf("no successful runs")
	}
	red, err := n.reduce(iters)
	if err != nil {
		return nil, nil, nil, nil, err
	}
	interMiss, unionMiss := make([][]string, len(failedIters)), make([][]string, len(failedIters))
	for i, f := range failedIters {
		if interMiss[i], err = n.missingFrom(red.inter, f); err != nil {
			return nil, nil, nil, nil, err
		}
		if unionMiss[i], err = n.missingFrom(red.union, f); err != nil {
			return nil, nil, nil, nil, err
		}
	}
	return codeWrap(n.tableNames(red.inter)), interMiss, codeWrap(n.tableNames(red.union)), unionMiss, nil
}

// ---- differential-provenance.go -------------------------------------------------------

// CreateNaiveDiffProv (differential-provenance.go:18-243): nemo_diffprov in
// NEMO_DIFF_REFERENCE (the in-place ###RUN### substitution of :43; the node
// context broadcasts failedRuns[0]'s label set to every device), the D masks,
// the missing rules (Missing.Goals = all D-children of each, the `leaf`
// rebinding of :93-95), the D edges (Q24) and the failed run's edges, then
// createDiffDot (unchanged).  `symmetric` is unused, as in the reference.
func (n *Neo4J) CreateNaiveDiffProv(symmetric bool, failedRuns []uint, successPostProv *gographviz.Graph) ([]*gographviz.Graph, []*gographviz.Graph, [][]*fi.Missing, error) {
	f := make([]C.uint32_t, len(failedRuns)+1)
	for i, it := range failedRuns {
		f[i] = C.uint32_t(it)
	}
	if err := n.err(C.nemo_diffprov(n.ctx, &f[0], C.size_t(len(failedRuns)), C.NEMO_DIFF_REFERENCE)); err != nil {
		return nil, nil, nil, err
	}
	g0 := 2*n.runIdx[0] + 1
	V0 := n.graphs[g0].n()
	var masks *C.uint8_t
	var ne, v0 C.uint64_t
	if err := n.err(C.nemo_diff_masks_view(n.ctx, &masks, &ne, &v0)); err != nil {
		return nil, nil, nil, err
	}
	maskOf := func(e int) []uint8 {
		return unsafe.Slice((*uint8)(unsafe.Pointer(masks)), int(ne)*V0)[e*V0 : (e+1)*V0]
	}
	var cnt C.uint64_t
	if err := n.err(C.nemo_fetch_missing(n.ctx, nil, 0, &cnt)); err != nil {
		return nil, nil, nil, err
	}
	rows := make([]C.nemo_missing, cnt+1)
	if err := n.err(C.nemo_fetch_missing(n.ctx, &rows[0], cnt, &cnt)); err != nil {
		return nil, nil, nil, err
	}
	// D-children of every missing rule from run 0's post edges (the interned arrays)
	children := n.childrenOf(g0)
	fl, err := n.flags(g0)
	if err != nil {
		return nil, nil, nil, err
	}
	missing := make([][]*fi.Missing, len(failedRuns))
	for _, row := range rows[:cnt] {
		e, rule := int(row.entry), uint32(row.rule)
		run := 2000 + failedRuns[e]
		rn := n.node(g0, rule, fl, &run)
		m := &fi.Missing{Rule: ruleOf(rn)}
		for _, ch := range children[rule] {
			if maskOf(e)[ch] != 0 {
				gn := n.node(g0, ch, fl, &run)
				m.Goals = append(m.Goals, goalOf(gn))
			}
		}
		missing[e] = append(missing[e], m)
	}
	if err := n.err(C.nemo_pull_edges(n.ctx, 2)); err != nil {
		return nil, nil, nil, err
	}
	diffEdges := make([][]graph.Path, len(failedRuns))
	for e, it := range failedRuns {
		run := 2000 + it
		if diffEdges[e], err = n.paths(uint32(e), g0, &run); err != nil {
			return nil, nil, nil, err
		}
	}
	diffDots, failedDots := make([]*gographviz.Graph, len(failedRuns)), make([]*gographviz.Graph, len(failedRuns))
	for e, it := range failedRuns {
		gf := 2*n.runIdx[it] + 1
		failedRows, err := n.rawPaths(gf)
		if err != nil {
			return nil, nil, nil, err
		}
		diffDots[e], failedDots[e], err = createDiffDot(2000+it, diffEdges[e], it, failedRows, 0,
			successPostProv, missing[e])
		if err != nil {
			return nil, nil, nil, err
		}
	}
	return diffDots, failedDots, missing, nil
}

func (n *Neo4J) childrenOf(g int) map[uint32][]uint32 {
	s, d := n.graphs[g].src, n.graphs[g].dst
	ch := map[uint32][]uint32{}
	for i := range s {
		ch[s[i]] = append(ch[s[i]], d[i])
	}
	for k := range ch {
		sort.Slice(ch[k], func(a, b int) bool { return ch[k][a] < ch[k][b] })
	}
	return ch
}

func goalOf(nd graph.Node) *fi.Goal {
	p := nd.Properties
	return &fi.Goal{ID: p["id"].(string), Label: p["label"].(string), Table: p["table"].(string),
		Time: p["time"].(string), CondHolds: p["condition_holds"] == true}
}

func ruleOf(nd graph.Node) *fi.Rule {
	p := nd.Properties
	return &fi.Rule{ID: p["id"].(string), Label: p["label"].(string), Table: p["table"].(string),
		Type: p["type"].(string)}
}

// ---- corrections.go / extensions.go ---------------------------------------------------

type triggerRows struct {
	pre   [][3]uint32 // (a, g, r) of findPreTriggers (corrections.go:30-34)
	post  [][2]uint32 // (g, r) of findPostTriggers (:121-125)
	async []uint32    // async rules of GenerateExtensions (extensions.go:63-67)
}

func (n *Neo4J) triggers() (*triggerRows, error) {
	if err := n.err(C.nemo_triggers(n.ctx)); err != nil {
		return nil, err
	}
	var np, nq, na C.uint64_t
	if err := n.err(C.nemo_fetch_triggers(n.ctx, nil, 0, &np, nil, 0, &nq, nil, 0, &na)); err != nil {
		return nil, err
	}
	pre, post, asy := make([]C.uint32_t, 3*np+1), make([]C.uint32_t, 2*nq+1), make([]C.uint32_t, na+1)
	if err := n.err(C.nemo_fetch_triggers(n.ctx, &pre[0], np, &np, &post[0], nq, &nq, &asy[0], na, &na)); err != nil {
		return nil, err
	}
	t := &triggerRows{}
	for i := 0; i < int(np); i++ {
		t.pre = append(t.pre, [3]uint32{uint32(pre[3*i]), uint32(pre[3*i+1]), uint32(pre[3*i+2])})
	}
	for i := 0; i < int(nq); i++ {
		t.post = append(t.post, [2]uint32{uint32(post[2*i]), uint32(post[2*i+1])})
	}
	for i := 0; i < int(na); i++ {
		t.async = append(t.async, uint32(asy[i]))
	}
	return t, nil
}

// receiver: strings.TrimLeft(label, table) -- a cutset trim -- then Trim "()"
// and the first ", " field (corrections.go:65-67,155-157).
func receiver(label, table string) string {
	return strings.Split(strings.Trim(strings.TrimLeft(label, table), "()"), ", ")[0]
}

// GenerateCorrections (corrections.go:202-328): the trigger rows of run 0 come
// from the device; the maps findPreTriggers / findPostTriggers returned are
// rebuilt with one fresh key per row (:76,168) and fed to the reference's own
// string synthesis (:219-324, kept verbatim as synthesizeCorrections).
func (n *Neo4J) GenerateCorrections() ([]string, error) {
	t, err := n.triggers()
	if err != nil {
		return nil, err
	}
	r0 := n.runIdx[0]
	gp, gq := 2*r0, 2*r0+1
	flp, err := n.flags(gp)
	if err != nil {
		return nil, err
	}
	flq, err := n.flags(gq)
	if err != nil {
		return nil, err
	}
	preTriggers := map[*fi.Rule][]*GoalRulePair{}
	for _, row := range t.pre {
		goal := goalOf(n.node(gp, row[1], flp, nil))
		goal.Receiver = receiver(goal.Label, goal.Table)
		agg := ruleOf(n.node(gp, row[0], flp, nil))
		preTriggers[agg] = append(preTriggers[agg], &GoalRulePair{Goal: goal, Rule: ruleOf(n.node(gp, row[2], flp, nil))})
	}
	postTriggers := map[*fi.Goal][]*fi.Rule{}
	for _, row := range t.post {
		goal := goalOf(n.node(gq, row[0], flq, nil))
		goal.Receiver = receiver(goal.Label, goal.Table)
		postTriggers[goal] = append(postTriggers[goal], ruleOf(n.node(gq, row[1], flq, nil)))
	}
	return synthesizeCorrections(preTriggers, postTriggers), nil
}

// GenerateExtensions (extensions.go:13-99): the holding-"pre" goal count is
// entry 2T+2 of the reduction vector (every shard's count summed);
// allAchievedPre = !(count < len(Runs)) (:47-49).
func (n *Neo4J) GenerateExtensions() (bool, []string, error) {
	red := n.red
	if red == nil {
		var err error
		if red, err = n.reduce(nil); err != nil {
			return false, nil, err
		}
	}
	if !(red.preHolds < uint64(len(n.Runs))) {
		return true, nil, nil
	}
	t, err := n.triggers()
	if err != nil {
		return false, nil, err
	}
	gp := 2 * n.runIdx[0]
	fl, err := n.flags(gp)
	if err != nil {
		return false, nil, err
	}
	state := map[string]string{}
	for _, r := range t.async { // one suggestion per distinct table (:83-90)
		table := n.node(gp, r, fl, nil).Properties["table"].(string)
		state[table] = fmt.Sprintf("<code>%s(node, ...)@async :- ...;</code>", table)
	}
	ext := make([]string, 0, len(state))
	for _, s := range state {
		ext = append(ext, s)
	}
	return false, ext, nil
}
