"""Server-side helpers shared by routers and services (reference ``server/utils``)."""
