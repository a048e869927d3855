// TEST INFRASTRUCTURE ONLY: a ~60-line stand-in for mocha (absent here) that runs the
// reference's own known-answer specs (packages/dds/merge-tree/src/test/*.spec.ts) after
// oracle/build_ref.py has transpiled them into oracle/_ref/.  It proves the transpiled
// reference behaves like the reference before it is trusted to make golden vectors.
// Usage: node oracle/run_ref_specs.mjs <spec module path>...
import path from "path";

const ctx = { timeout() { return ctx; }, slow() { return ctx; }, skip() {} };
let current = { name: "", tests: [], before: [], beforeEach: [], afterEach: [], children: [] };
const root = current;
globalThis.describe = (name, fn) => {
    const s = { name, tests: [], before: [], beforeEach: [], afterEach: [], children: [], parent: current };
    current.children.push(s);
    const prev = current;
    current = s;
    fn.call(ctx);
    current = prev;
};
globalThis.describe.skip = () => {};
globalThis.describe.only = globalThis.describe;
globalThis.it = (name, fn) => { current.children.push({ name, fn, test: true }); return ctx; };
globalThis.it.skip = (name) => { current.children.push({ name, skip: true, test: true }); };
globalThis.it.only = globalThis.it;
globalThis.before = (fn) => current.before.push(fn);
globalThis.beforeEach = (fn) => current.beforeEach.push(fn);
globalThis.afterEach = (fn) => current.afterEach.push(fn);
globalThis.after = () => {};

let passed = 0, failed = 0, skipped = 0;
async function run(s, prefix, hooks) {
    for (const b of s.before || []) { await b.call(ctx); }
    const be = hooks.beforeEach.concat(s.beforeEach || []);
    const ae = (s.afterEach || []).concat(hooks.afterEach);
    for (const c of s.children) {
        if (c.test) {
            const name = `${prefix} ${c.name}`;
            if (c.skip) { skipped++; continue; }
            try {
                for (const b of be) { await b(); }
                await c.fn.call(ctx);
                for (const a of ae) { await a(); }
                passed++;
            } catch (e) {
                failed++;
                console.log(`FAIL ${name}: ${e && e.message ? e.message.split("\n")[0] : e}`);
            }
        } else {
            await run(c, `${prefix} ${c.name}`, { beforeEach: be, afterEach: ae });
        }
    }
}

(async () => {
    for (const f of process.argv.slice(2)) {
        await import(path.resolve(f));
    }
    await run(root, "", { beforeEach: [], afterEach: [] });
    console.log(JSON.stringify({ passed, failed, skipped }));
    process.exit(failed ? 1 : 0);
})().catch((e) => { console.log("ERROR", e && e.stack); process.exit(2); });
