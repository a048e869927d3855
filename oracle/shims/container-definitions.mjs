// TEST INFRASTRUCTURE ONLY: AttachState enum of @fluidframework/container-definitions.
export const AttachState = { Detached: "Detached", Attaching: "Attaching", Attached: "Attached" };
