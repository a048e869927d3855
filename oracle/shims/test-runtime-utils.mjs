// TEST INFRASTRUCTURE ONLY: MockStorage restated from
// packages/runtime/test-runtime-utils/src/mockStorage.ts:15-53 (read blobs out of an ITree).
function readCore(tree, paths) {
    if (!tree) { return undefined; }
    for (const entry of tree.entries) {
        if (entry.path === paths[0]) {
            if (entry.type === "Blob") {
                return Buffer.from(entry.value.contents, entry.value.encoding || "utf8").toString("base64");
            }
            if (entry.type === "Tree") { return readCore(entry.value, paths.slice(1)); }
            return undefined;
        }
    }
    return undefined;
}
export class MockStorage {
    constructor(tree) { this.tree = tree; }
    async read(path) {
        const blob = readCore(this.tree, path.split("/"));
        if (blob === undefined) { throw new Error(`Blob does not exist: ${path}`); }
        return blob;
    }
    async contains(path) { return readCore(this.tree, path.split("/")) !== undefined; }
    // listBlobsAtTreePath: packages/runtime/runtime-utils/src/objectstorageutils.ts:22-46
    async list(path) {
        const parts = path.split("/").filter((p) => p.length > 0);
        let tree = this.tree;
        while (tree && tree.entries !== undefined && parts.length > 0) {
            const part = parts.shift();
            const e = tree.entries.find((v) => v.type === "Tree" && v.path === part);
            tree = e ? e.value : undefined;
        }
        if (!tree || tree.entries === undefined || parts.length !== 0) { throw new Error("path does not exist"); }
        return tree.entries.filter((e) => e.type === "Blob").map((e) => e.path);
    }
}
